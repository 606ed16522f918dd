// xml_bsdf.cpp -- the BSDF subtrees of a Mitsuba 0.6 scene file for the
// plugin shim (integration/gpupath.cpp).
//
// Inside Mitsuba, `twosided` keeps its nested BSDFs and every BSDF keeps its
// textures as private children (src/bsdfs/twosided.cpp:198-210, the
// Texture-valued members of diffuse/rough*.cpp): a plugin cannot reach them.
// The scene's source file can (Scene::getSourceFile,
// include/mitsuba/render/scene.h:1107).  mtsgpu_xml_bsdf reads that file and
// returns the element tree below the BSDF with the requested id -- nested
// <bsdf> and <texture> elements, <ref> children resolved by id, and the
// property elements of each with `$name` defaults substituted -- as flat
// arrays.  The shim turns each node back into a Properties object and converts
// it with the code it uses for the BSDFs it can see.
//
// The XML subset is the scene format's own (SceneHandler, src/librender/
// scenehandler.cpp): elements, attributes in single or double quotes,
// self-closing tags, comments, the XML declaration, the five predefined
// entities.  <include> is not followed.
#include <cstdio>
#include <cstring>
#include <fstream>
#include <map>
#include <memory>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/mtsgpu.h"

namespace {

struct XElem {
    std::string tag;
    std::vector<std::pair<std::string, std::string>> attrs;
    std::vector<std::unique_ptr<XElem>> kids;
    const std::string *attr(const char *k) const {
        for (auto &a : attrs)
            if (a.first == k) return &a.second;
        return nullptr;
    }
};

struct XParser {
    const std::string &s;
    size_t i = 0;
    std::string err;
    explicit XParser(const std::string &src) : s(src) {}

    bool fail(const std::string &m) {
        if (err.empty()) {
            size_t line = 1;
            for (size_t k = 0; k < i && k < s.size(); ++k) line += s[k] == '\n';
            err = m + " (line " + std::to_string(line) + ")";
        }
        return false;
    }
    void ws() {
        while (i < s.size() && (s[i] == ' ' || s[i] == '\t' || s[i] == '\n' || s[i] == '\r')) ++i;
    }
    bool starts(const char *p) const { return s.compare(i, std::strlen(p), p) == 0; }
    // skips comments, declarations, processing instructions and text up to the next element tag
    bool skip_misc() {
        while (i < s.size()) {
            if (starts("<!--")) {
                const size_t e = s.find("-->", i + 4);
                if (e == std::string::npos) return fail("unterminated comment");
                i = e + 3;
            } else if (starts("<?") || starts("<!")) {
                const size_t e = s.find('>', i);
                if (e == std::string::npos) return fail("unterminated declaration");
                i = e + 1;
            } else if (s[i] == '<') {
                return true;
            } else {
                ++i;   // character data: the scene format has none that matters
            }
        }
        return true;
    }
    static std::string unescape(const std::string &v) {
        std::string o;
        for (size_t k = 0; k < v.size(); ++k) {
            if (v[k] == '&') {
                static const char *ent[5][2] = {{"&lt;", "<"}, {"&gt;", ">"}, {"&amp;", "&"}, {"&quot;", "\""}, {"&apos;", "'"}};
                bool hit = false;
                for (auto &e : ent)
                    if (v.compare(k, std::strlen(e[0]), e[0]) == 0) { o += e[1]; k += std::strlen(e[0]) - 1; hit = true; break; }
                if (!hit) o += v[k];
            } else {
                o += v[k];
            }
        }
        return o;
    }
    std::string name() {
        const size_t b = i;
        while (i < s.size() && (isalnum((unsigned char)s[i]) || s[i] == '_' || s[i] == '-' || s[i] == ':' || s[i] == '.')) ++i;
        return s.substr(b, i - b);
    }
    // an element starting at '<' (not a closing tag)
    bool element(XElem &e) {
        ++i;   // '<'
        e.tag = name();
        if (e.tag.empty()) return fail("expected an element name");
        while (true) {
            ws();
            if (i >= s.size()) return fail("unterminated tag <" + e.tag + ">");
            if (starts("/>")) { i += 2; return true; }
            if (s[i] == '>') { ++i; break; }
            std::string k = name();
            if (k.empty()) return fail("bad attribute in <" + e.tag + ">");
            ws();
            if (i >= s.size() || s[i] != '=') return fail("expected '=' after attribute " + k);
            ++i;
            ws();
            if (i >= s.size() || (s[i] != '"' && s[i] != '\'')) return fail("expected a quoted value for " + k);
            const char q = s[i++];
            const size_t e2 = s.find(q, i);
            if (e2 == std::string::npos) return fail("unterminated attribute value");
            e.attrs.emplace_back(k, unescape(s.substr(i, e2 - i)));
            i = e2 + 1;
        }
        while (true) {   // children up to </tag>
            if (!skip_misc()) return false;
            if (i >= s.size()) return fail("missing </" + e.tag + ">");
            if (starts("</")) {
                i += 2;
                const std::string t = name();
                ws();
                if (t != e.tag || i >= s.size() || s[i] != '>') return fail("mismatched </" + t + "> for <" + e.tag + ">");
                ++i;
                return true;
            }
            e.kids.emplace_back(new XElem());
            if (!element(*e.kids.back())) return false;
        }
    }
    bool document(XElem &root) {
        if (!skip_misc()) return false;
        if (i >= s.size()) return fail("no root element");
        return element(root);
    }
};

struct TreeBuilder {
    const XElem &root;
    std::map<std::string, const XElem *> ids;
    std::map<std::string, std::string> defaults;
    std::vector<mtsgpu_xml_node> nodes;
    std::vector<mtsgpu_xml_prop> props;
    std::string err;

    explicit TreeBuilder(const XElem &r) : root(r) {
        index(root);
        for (auto &k : root.kids)
            if (k->tag == "default" && k->attr("name") && k->attr("value")) defaults[*k->attr("name")] = *k->attr("value");
    }
    void index(const XElem &e) {
        if (const std::string *id = e.attr("id"))
            if (e.tag != "scene" && !ids.count(*id)) ids[*id] = &e;
        for (auto &k : e.kids) index(*k);
    }
    // $name -> its <default> value (the loader's -D parameters are not known here)
    bool subst(const std::string &v, std::string &out) {
        out.clear();
        for (size_t k = 0; k < v.size(); ++k) {
            if (v[k] != '$') { out += v[k]; continue; }
            size_t e = k + 1;
            while (e < v.size() && (isalnum((unsigned char)v[e]) || v[e] == '_')) ++e;
            const std::string n = v.substr(k + 1, e - k - 1);
            auto it = defaults.find(n);
            if (n.empty() || it == defaults.end()) { err = "unresolved parameter $" + n + " (no <default>)"; return false; }
            out += it->second;
            k = e - 1;
        }
        return true;
    }
    static bool copy(char *dst, size_t cap, const std::string &v) {
        if (v.size() + 1 > cap) return false;
        std::memcpy(dst, v.c_str(), v.size() + 1);
        return true;
    }
    bool node(const XElem &e, int parent, const std::string &pname, int depth) {
        if (depth > 16) { err = "BSDF references nest too deeply (a <ref> cycle?)"; return false; }
        mtsgpu_xml_node n;
        std::memset(&n, 0, sizeof n);
        n.kind = e.tag == "bsdf" ? MTSGPU_XML_BSDF : MTSGPU_XML_TEXTURE;
        n.parent = parent;
        const std::string *type = e.attr("type");
        if (!type) { err = "<" + e.tag + "> without a type"; return false; }
        const std::string *id = e.attr("id");
        if (!copy(n.plugin, sizeof n.plugin, *type) || !copy(n.name, sizeof n.name, pname) ||
            !copy(n.id, sizeof n.id, id ? *id : std::string())) {
            err = "name too long in <" + e.tag + " type=\"" + *type + "\">";
            return false;
        }
        const int self = (int)nodes.size();
        nodes.push_back(n);
        // property elements first (they are the node's own), then the children
        nodes[self].first_prop = (int)props.size();
        for (auto &k : e.kids) {
            const std::string &t = k->tag;
            if (t == "bsdf" || t == "texture" || t == "ref") continue;
            mtsgpu_xml_prop p;
            std::memset(&p, 0, sizeof p);
            const std::string *nm = k->attr("name");
            std::string val;
            const std::string *v = k->attr("value");
            if (v && !subst(*v, val)) return false;
            if (!v && (t == "point" || t == "vector")) {   // x/y/z form
                std::string x, y, z;
                if (!subst(k->attr("x") ? *k->attr("x") : "0", x) || !subst(k->attr("y") ? *k->attr("y") : "0", y) ||
                    !subst(k->attr("z") ? *k->attr("z") : "0", z))
                    return false;
                val = x + ", " + y + ", " + z;
            } else if (!v) {
                err = "<" + t + "> in <" + e.tag + " type=\"" + *type + "\"> has no value (not supported here)";
                return false;
            }
            if (!copy(p.tag, sizeof p.tag, t) || !copy(p.name, sizeof p.name, nm ? *nm : std::string()) ||
                !copy(p.value, sizeof p.value, val)) {
                err = "property too long in <" + e.tag + " type=\"" + *type + "\">";
                return false;
            }
            props.push_back(p);
        }
        nodes[self].num_props = (int)props.size() - nodes[self].first_prop;
        for (auto &k : e.kids) {
            const std::string &t = k->tag;
            const std::string *nm = k->attr("name");
            const std::string cname = nm ? *nm : std::string();
            if (t == "bsdf" || t == "texture") {
                if (!node(*k, self, cname, depth + 1)) return false;
            } else if (t == "ref") {
                const std::string *rid = k->attr("id");
                auto it = rid ? ids.find(*rid) : ids.end();
                if (it == ids.end()) { err = "Unable to find object with id \"" + (rid ? *rid : std::string()) + "\""; return false; }
                if (it->second->tag != "bsdf" && it->second->tag != "texture") {
                    err = "<ref id=\"" + *rid + "\"> in a BSDF names a <" + it->second->tag + ">";
                    return false;
                }
                if (!node(*it->second, self, cname, depth + 1)) return false;
            }
        }
        return true;
    }
};

}  // namespace

extern "C" int mtsgpu_xml_bsdf(const char *xml_path, const char *bsdf_id, mtsgpu_xml_node *nodes, int node_cap,
                               mtsgpu_xml_prop *props, int prop_cap, int *num_nodes, int *num_props, char *err,
                               size_t err_cap) {
    auto fail = [&](int code, const std::string &m) {
        if (err && err_cap) {
            std::snprintf(err, err_cap, "%s", m.c_str());
        }
        return code;
    };
    if (!xml_path || !bsdf_id || !num_nodes || !num_props || node_cap < 0 || prop_cap < 0)
        return fail(MTSGPU_EINVAL, "null argument");
    *num_nodes = *num_props = 0;
    std::ifstream f(xml_path, std::ios::binary);
    if (!f) return fail(MTSGPU_EINVAL, std::string("cannot read ") + xml_path);
    std::stringstream ss;
    ss << f.rdbuf();
    const std::string src = ss.str();
    XElem root;
    XParser P(src);
    if (!P.document(root)) return fail(MTSGPU_EINVAL, std::string(xml_path) + ": " + P.err);
    TreeBuilder E(root);
    auto it = E.ids.find(bsdf_id);
    if (it == E.ids.end() || it->second->tag != "bsdf")
        return fail(MTSGPU_EINVAL, std::string("no <bsdf id=\"") + bsdf_id + "\"> in " + xml_path);
    if (!E.node(*it->second, -1, std::string(), 0)) return fail(MTSGPU_EINVAL, E.err);
    *num_nodes = (int)E.nodes.size();
    *num_props = (int)E.props.size();
    if ((int)E.nodes.size() > node_cap || (int)E.props.size() > prop_cap)
        return fail(MTSGPU_ENOMEM, "node or property capacity too small (counts returned)");
    if (nodes) std::memcpy(nodes, E.nodes.data(), E.nodes.size() * sizeof(mtsgpu_xml_node));
    if (props) std::memcpy(props, E.props.data(), E.props.size() * sizeof(mtsgpu_xml_prop));
    return MTSGPU_OK;
}
