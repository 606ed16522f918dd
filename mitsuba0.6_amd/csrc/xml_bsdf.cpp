// xml_bsdf.cpp -- the BSDF subtrees of a Mitsuba 0.6 scene file for the
// plugin shim (integration/gpupath.cpp).
//
// Inside Mitsuba, `twosided` keeps its nested BSDFs and every BSDF keeps its
// textures as private children (src/bsdfs/twosided.cpp:198-210, the
// Texture-valued members of diffuse/rough*.cpp): a plugin cannot reach them.
// The scene's source file can (Scene::getSourceFile,
// include/mitsuba/render/scene.h:1107).  mtsgpu_xml_bsdf_ex reads that file
// and returns the element tree below a BSDF -- nested <bsdf> and <texture>
// elements, <ref> children resolved by id, and the property elements of each
// -- as flat arrays.  The shim turns each node back into a Properties object
// and converts it with the code it uses for the BSDFs it can see.
//
// The file is read as SceneHandler reads it (src/librender/scenehandler.cpp):
//   - every attribute of every element has its $parameters replaced when the
//     element starts (:208-220): the loader's parameters (the caller's list, e.g.
//     the `mitsuba -D name=value` map, src/mitsuba/mitsuba.cpp:168-173) in
//     reverse name order, by plain substring replacement; a '$' left over
//     without a '[' is an error;
//   - <default name value> adds a parameter when the element ends, unless the
//     loader already has it (:684-687), so the caller's values win;
//   - ids are registered when their element ends; a second element with the
//     same id is an error (:784-786), and so is an <alias> onto a taken id
//     (:646-656);
//   - <include filename> parses the named file with the ids shared and a copy
//     of the parameters (:658-680, SceneHandler(m_params, ...)), so a <default>
//     inside the included file does not reach the including one; a relative
//     name resolves against the main scene file's directory first, as the
//     FileResolver has it first (mitsuba.cpp), then as given;
//   - the `type` attribute is lower-cased (:275).
// Each returned property carries flags saying whether its value went through a
// substitution and whether a <default> supplied it, so a caller that cannot
// see the loader's parameters can check those values against the plugin's own.
//
// The XML subset is the scene format's own: elements, attributes in single or
// double quotes, self-closing tags, comments, the XML declaration, the five
// predefined entities.
#include <sys/stat.h>

#include <cctype>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/mtsgpu.h"

namespace {

struct XElem {
    std::string tag;
    std::vector<std::pair<std::string, std::string>> attrs;
    std::vector<int> flags;   // per attribute: MTSGPU_XML_PROP_* after expansion
    std::vector<std::unique_ptr<XElem>> kids;
    int line = 0;
    const std::string *attr(const char *k) const {
        for (auto &a : attrs)
            if (a.first == k) return &a.second;
        return nullptr;
    }
    int attr_flags(const char *k) const {
        for (size_t j = 0; j < attrs.size(); ++j)
            if (attrs[j].first == k) return j < flags.size() ? flags[j] : 0;
        return 0;
    }
};

struct XParser {
    const std::string &s;
    size_t i = 0;
    std::string err;
    explicit XParser(const std::string &src) : s(src) {}

    // line numbers: counted forward from the last position asked for (elements are
    // parsed in document order), so a parse is linear in the file size
    size_t line_pos = 0;
    int line_no = 1;
    int line_at(size_t pos) {
        if (pos < line_pos) { line_pos = 0; line_no = 1; }
        for (; line_pos < pos && line_pos < s.size(); ++line_pos) line_no += s[line_pos] == '\n';
        return line_no;
    }
    bool fail(const std::string &m) {
        if (err.empty()) err = m + " (line " + std::to_string(line_at(i)) + ")";
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
        e.line = line_at(i);
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

bool read_file(const std::string &path, std::string &out) {
    std::ifstream f(path, std::ios::binary);
    if (!f) return false;
    std::stringstream ss;
    ss << f.rdbuf();
    out = ss.str();
    return true;
}

std::string dir_of(const std::string &path) {
    const size_t k = path.find_last_of('/');
    return k == std::string::npos ? std::string() : path.substr(0, k + 1);
}

// The document-order pass of SceneHandler over a file and its includes:
// parameter substitution, <default>, ids, <alias>, <include>.
bool file_exists(const std::string &path) {
    struct stat st;
    return ::stat(path.c_str(), &st) == 0;
}

struct Loader {
    std::map<std::string, std::string> params;   // name -> value (the loader's and then <default>'s)
    std::set<std::string> from_default;          // names a <default> supplied
    std::map<std::string, const XElem *> ids;
    std::vector<std::unique_ptr<XElem>> roots;   // the main file and every included file
    std::vector<std::string> files;
    std::string err;

    bool fail(const std::string &file, const XElem &e, const std::string &m) {
        if (err.empty()) err = file + " (line " + std::to_string(e.line) + "): " + m;
        return false;
    }
    // scenehandler.cpp:208-220, with a record of where the replacements came from
    bool subst(std::string &v, int &flags) {
        flags = 0;
        if (v.empty() || v.find('$') == std::string::npos) return true;
        for (auto it = params.rbegin(); it != params.rend(); ++it) {
            const std::string search = "$" + it->first;
            size_t pos = 0;
            while ((pos = v.find(search, pos)) != std::string::npos) {
                v.replace(pos, search.size(), it->second);
                flags |= MTSGPU_XML_PROP_PARAM | (from_default.count(it->first) ? MTSGPU_XML_PROP_DEFAULT : 0);
                ++pos;
            }
        }
        return v.find('$') == std::string::npos || v.find('[') != std::string::npos;
    }
    bool load(const std::string &path, int depth) {
        if (depth > 16) { err = path + ": <include> nests too deeply"; return false; }
        std::string src;
        if (!read_file(path, src)) { err = "cannot read " + path; return false; }
        std::unique_ptr<XElem> root(new XElem());
        XParser P(src);
        if (!P.document(*root)) { err = path + ": " + P.err; return false; }
        XElem *r = root.get();
        roots.push_back(std::move(root));
        files.push_back(path);
        return walk(*r, path, depth);
    }
    bool walk(XElem &e, const std::string &file, int depth) {
        e.flags.assign(e.attrs.size(), 0);
        for (size_t j = 0; j < e.attrs.size(); ++j)      // startElement
            if (!subst(e.attrs[j].second, e.flags[j]))
                return fail(file, e, "The scene referenced an undefined parameter: \"" + e.attrs[j].second + "\"");
        for (auto &a : e.attrs)
            if (a.first == "type")
                for (auto &c : a.second) c = (char)std::tolower((unsigned char)c);
        for (auto &k : e.kids)
            if (!walk(*k, file, depth)) return false;
        // endElement
        if (e.tag == "default") {
            const std::string *n = e.attr("name"), *v = e.attr("value");
            if (n && v && !params.count(*n)) {
                params[*n] = *v;
                from_default.insert(*n);
            }
            return true;
        }
        if (e.tag == "alias") {
            const std::string *id = e.attr("id"), *as = e.attr("as");
            auto it = id ? ids.find(*id) : ids.end();
            if (it == ids.end()) return fail(file, e, "Referenced object '" + (id ? *id : std::string()) + "' not found!");
            if (!as || ids.count(*as)) return fail(file, e, "Duplicate ID '" + *id + "' used in scene description!");
            ids[*as] = it->second;
            return true;
        }
        if (e.tag == "include") {
            const std::string *fn = e.attr("filename");
            if (!fn) return fail(file, e, "<include> without a filename");
            std::string p = *fn;
            if (!fn->empty() && (*fn)[0] != '/' && file_exists(dir_of(files[0]) + *fn)) p = dir_of(files[0]) + *fn;
            // SceneHandler(m_params, m_namedObjects, true): ids shared, parameters copied
            const std::map<std::string, std::string> saved = params;
            const std::set<std::string> savedDefault = from_default;
            const bool ok = load(p, depth + 1);
            params = saved;
            from_default = savedDefault;
            return ok;
        }
        const std::string *id = e.attr("id");
        if (id && !id->empty() && e.tag != "ref" && e.tag != "scene") {
            if (ids.count(*id)) return fail(file, e, "Duplicate ID '" + *id + "' used in scene description!");
            ids[*id] = &e;
        }
        return true;
    }
};

struct TreeBuilder {
    const Loader &L;
    std::vector<mtsgpu_xml_node> nodes;
    std::vector<mtsgpu_xml_prop> props;
    std::string err;

    explicit TreeBuilder(const Loader &l) : L(l) {}
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
            if (v) {
                val = *v;
                p.flags = k->attr_flags("value");
                // a sampled spectrum ("wavelength:value, ..."): the plugin's parsed value is used
                if (t == "spectrum" && val.find(':') != std::string::npos) p.flags |= MTSGPU_XML_PROP_UNSUPPORTED;
            } else if (t == "point" || t == "vector") {   // x/y/z form
                auto xyz = [&](const char *a) { return k->attr(a) ? *k->attr(a) : std::string("0"); };
                val = xyz("x") + ", " + xyz("y") + ", " + xyz("z");
                p.flags = k->attr_flags("x") | k->attr_flags("y") | k->attr_flags("z");
            } else {
                // <spectrum filename=...>, <blackbody temperature=...>, ...: the attributes as
                // text; the caller takes the value from the plugin's own Properties
                for (size_t a = 0; a < k->attrs.size(); ++a) {
                    if (k->attrs[a].first == "name") continue;
                    if (!val.empty()) val += " ";
                    val += k->attrs[a].first + "=" + k->attrs[a].second;
                    p.flags |= k->flags[a];
                }
                if (val.size() > sizeof p.value - 1) val.resize(sizeof p.value - 1);
                p.flags |= MTSGPU_XML_PROP_UNSUPPORTED;
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
                const XElem *r = resolve(*k);
                if (!r) return false;
                if (r->tag != "bsdf" && r->tag != "texture") {
                    err = "<ref id=\"" + *k->attr("id") + "\"> in a BSDF names a <" + r->tag + ">";
                    return false;
                }
                if (!node(*r, self, cname, depth + 1)) return false;
            }
        }
        return true;
    }
    const XElem *resolve(const XElem &ref) {
        const std::string *rid = ref.attr("id");
        auto it = rid ? L.ids.find(*rid) : L.ids.end();
        if (it == L.ids.end()) {
            err = "Referenced object '" + (rid ? *rid : std::string()) + "' not found!";
            return nullptr;
        }
        return it->second;
    }
};

// One parsed scene per (file, parameters), reused while none of its files changed
// (size and modification time of the main file and of every include): the shim asks
// once per BSDF, and an exported scene with thousands of shapes must not be re-read
// for each.
struct FileStamp {
    std::string path;
    long long size, mtime_ns;
    bool operator==(const FileStamp &o) const { return path == o.path && size == o.size && mtime_ns == o.mtime_ns; }
};
FileStamp stamp(const std::string &path) {
    struct stat st;
    if (::stat(path.c_str(), &st) != 0) return {path, -1, -1};
    return {path, (long long)st.st_size, (long long)st.st_mtim.tv_sec * 1000000000ll + st.st_mtim.tv_nsec};
}
struct CacheEntry {
    std::map<std::string, std::string> params;
    std::vector<FileStamp> stamps;
    std::shared_ptr<const Loader> loader;
};
std::mutex g_cache_mu;
std::vector<CacheEntry> g_cache;   // most recent last, at most 4 scenes

std::shared_ptr<const Loader> cached_load(const std::string &path, const std::map<std::string, std::string> &params,
                                          std::string &err) {
    std::lock_guard<std::mutex> lock(g_cache_mu);
    for (size_t k = 0; k < g_cache.size(); ++k) {
        const CacheEntry &c = g_cache[k];
        if (c.params != params || c.stamps.empty() || c.stamps[0].path != path) continue;
        bool same = true;
        for (const FileStamp &f : c.stamps) same = same && stamp(f.path) == f;
        if (same) return c.loader;
    }
    std::shared_ptr<Loader> L(new Loader());
    L->params = params;
    if (!L->load(path, 0)) {
        err = L->err;
        return nullptr;
    }
    CacheEntry c;
    c.params = params;
    for (const std::string &f : L->files) c.stamps.push_back(stamp(f));
    c.loader = L;
    if (g_cache.size() >= 4) g_cache.erase(g_cache.begin());
    g_cache.push_back(c);
    return L;
}

}  // namespace

extern "C" int mtsgpu_xml_bsdf_ex(const char *xml_path, const char *id, int32_t lookup, const char *const *param_names,
                                  const char *const *param_values, int32_t num_params, mtsgpu_xml_node *nodes,
                                  int node_cap, mtsgpu_xml_prop *props, int prop_cap, int *num_nodes, int *num_props,
                                  char *err, size_t err_cap) {
    auto fail = [&](int code, const std::string &m) {
        if (err && err_cap) std::snprintf(err, err_cap, "%s", m.c_str());
        return code;
    };
    if (!xml_path || !id || !num_nodes || !num_props || node_cap < 0 || prop_cap < 0 || num_params < 0 ||
        (num_params > 0 && (!param_names || !param_values)) ||
        (lookup != MTSGPU_XML_BY_ID && lookup != MTSGPU_XML_BY_SHAPE))
        return fail(MTSGPU_EINVAL, "null or invalid argument");
    *num_nodes = *num_props = 0;
    std::map<std::string, std::string> params;
    for (int k = 0; k < num_params; ++k) {
        if (!param_names[k] || !param_values[k]) return fail(MTSGPU_EINVAL, "null parameter name or value");
        params[param_names[k]] = param_values[k];
    }
    std::string lerr;
    std::shared_ptr<const Loader> Lp = cached_load(xml_path, params, lerr);
    if (!Lp) return fail(MTSGPU_EINVAL, lerr);
    const Loader &L = *Lp;
    TreeBuilder E(L);
    auto it = L.ids.find(id);
    const XElem *bsdf = nullptr;
    if (lookup == MTSGPU_XML_BY_ID) {
        if (it == L.ids.end()) return fail(MTSGPU_ENOENT, std::string("no element with id \"") + id + "\" in " + xml_path);
        if (it->second->tag != "bsdf")
            return fail(MTSGPU_EINVAL, std::string("id \"") + id + "\" names a <" + it->second->tag + ">, not a <bsdf>");
        bsdf = it->second;
    } else {
        // the BSDF given inline (or by <ref>) inside the <shape> with this id
        if (it == L.ids.end()) return fail(MTSGPU_ENOENT, std::string("no element with id \"") + id + "\" in " + xml_path);
        if (it->second->tag != "shape")
            return fail(MTSGPU_EINVAL, std::string("id \"") + id + "\" names a <" + it->second->tag + ">, not a <shape>");
        for (auto &k : it->second->kids) {
            const XElem *c = k.get();
            if (c->tag == "ref") {
                c = E.resolve(*c);
                if (!c) return fail(MTSGPU_EINVAL, E.err);
            }
            if (c->tag == "bsdf") {
                if (bsdf) return fail(MTSGPU_EINVAL, std::string("shape \"") + id + "\" has more than one BSDF");
                bsdf = c;
            }
        }
        if (!bsdf) return fail(MTSGPU_ENOENT, std::string("shape \"") + id + "\" has no <bsdf> in " + xml_path);
    }
    if (!E.node(*bsdf, -1, std::string(), 0)) return fail(MTSGPU_EINVAL, E.err);
    *num_nodes = (int)E.nodes.size();
    *num_props = (int)E.props.size();
    if ((int)E.nodes.size() > node_cap || (int)E.props.size() > prop_cap)
        return fail(MTSGPU_ENOMEM, "node or property capacity too small (counts returned)");
    if (nodes) std::memcpy(nodes, E.nodes.data(), E.nodes.size() * sizeof(mtsgpu_xml_node));
    if (props) std::memcpy(props, E.props.data(), E.props.size() * sizeof(mtsgpu_xml_prop));
    return MTSGPU_OK;
}

extern "C" int mtsgpu_xml_bsdf(const char *xml_path, const char *bsdf_id, mtsgpu_xml_node *nodes, int node_cap,
                               mtsgpu_xml_prop *props, int prop_cap, int *num_nodes, int *num_props, char *err,
                               size_t err_cap) {
    return mtsgpu_xml_bsdf_ex(xml_path, bsdf_id, MTSGPU_XML_BY_ID, nullptr, nullptr, 0, nodes, node_cap, props,
                              prop_cap, num_nodes, num_props, err, err_cap);
}
