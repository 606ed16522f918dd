/*
 * gpupath.cpp -- the reference-side plugin shim: `path`, `volpath` (no media)
 * and `direct` as Mitsuba 0.6 integrator plugins that render through
 * libmtsgpu.so (include/mtsgpu.h).
 *
 * A Mitsuba maintainer adds this file to src/integrators/ and builds it like
 * the other integrators (SConscript:
 *     plugins += env.SharedLibrary('gpupath', ['gpupath.cpp'], LIBS=env['LIBS'] + ['mtsgpu'])
 * with CPPPATH += <repo>/include and LIBPATH += <repo>/mitsuba0.6_amd/_build).
 * Three plugin names come out of one source by -DGPU_INTEGRATOR=<0|1|2>
 * (gpupath / gpuvolpath / gpudirect).  It is not compiled in this repository:
 * every Mitsuba header includes boost, which this image lacks.
 *
 * Reference interfaces this follows:
 *   plugin entry points       include/mitsuba/core/cobject.h:99-107 (MTS_EXPORT_PLUGIN),
 *                             loaded by src/libcore/plugin.cpp:62-123
 *   Integrator::render        include/mitsuba/render/integrator.h:74-75, the call that is replaced
 *   MonteCarloIntegrator      include/mitsuba/render/integrator.h:458-461 (maxDepth, rrDepth,
 *                             strictNormals, hideEmitters), parsed in integrator.cpp:190-225
 *   Film::put                 src/librender/renderproc.cpp:142-149 (how blocks reach the film)
 *   Integrator::cancel        integrator.h:88 (-> the library's cancel flag)
 *
 * Li() is the one per-ray entry point a whole-frame GPU renderer cannot serve
 * (E() / irradiance-cache callers, SamplingIntegrator::renderBlock users): it
 * delegates to the reference's own CPU integrator of the same name and
 * properties, created through the PluginManager, so such callers get exactly
 * the reference's behaviour.
 *
 * Multi-GPU: the 'devices' property ("0,1,2,3"; default: the current device)
 * selects a device group; mtsgpu_group_render shards the crop's 8x8 tiles
 * over the GPUs and merges the films over xGMI before Film::put.
 *
 * BSDFs: the plugins keep nested BSDFs (twosided) and textures as private
 * children, so the scene file is the authority.  Every BSDF the file holds --
 * by its own id, or inline in a <shape> with an id -- is read back from it
 * (Scene::getSourceFile, scene.h:1107) through mtsgpu_xml_bsdf_ex with the
 * loader's parameters, rebuilt as one Properties object per element and
 * converted like any other BSDF.  A BSDF the file does not hold is converted
 * from its Properties only when it is not twosided and shows no textured
 * parameter; otherwise the render stops with an error naming the shape.
 */
#include <mitsuba/render/scene.h>
#include <mitsuba/render/trimesh.h>
#include <mitsuba/render/renderjob.h>
#include <mitsuba/render/texture.h>
#include <mitsuba/core/plugin.h>
#include <mitsuba/core/fresolver.h>
#include <mitsuba/core/fstream.h>
#include <mitsuba/core/bitmap.h>

#include <cstring>
#include <set>
#include <vector>
#include <fstream>
#include <sstream>

#include "../bsdfs/ior.h"      /* lookupIOR: the BSDF plugins' IOR presets */
#include "mtsgpu.h"
#include "gpupath_util.h"

#ifndef GPU_INTEGRATOR
#define GPU_INTEGRATOR 0     /* 0: path, 1: volpath, 2: direct */
#endif

MTS_NAMESPACE_BEGIN

namespace {

const char *cpuPluginName() {
    return GPU_INTEGRATOR == 1 ? "volpath" : GPU_INTEGRATOR == 2 ? "direct" : "path";
}

template <class T> int indexOf(const std::vector<const T *> &v, const T *p) {
    for (size_t i = 0; i < v.size(); ++i)
        if (v[i] == p) return (int) i;
    return -1;
}

void toRGB(const Spectrum &s, float *rgb) {
    Float r, g, b;
    s.toLinearRGB(r, g, b);
    rgb[0] = (float) r; rgb[1] = (float) g; rgb[2] = (float) b;
}

void copyMatrix(const Matrix4x4 &m, float *out) {
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j)
            out[4 * i + j] = (float) m.m[i][j];
}

int distribution(const Properties &p) {    /* microfacet.h:104-115 */
    std::string d = p.getString("distribution", "beckmann");
    for (size_t i = 0; i < d.size(); ++i) d[i] = (char) tolower(d[i]);
    return d == "ggx" ? MTSGPU_DISTR_GGX : (d == "phong" || d == "as") ? MTSGPU_DISTR_PHONG : MTSGPU_DISTR_BECKMANN;
}

/* The bytes of data/microfacet/<distr>.dat as RoughTransmittance reads them
   (rtrans.h:46-150, through the FileResolver) */
const std::vector<char> &rtransBytes(int distr) {
    static std::vector<char> cache[3];
    std::vector<char> &b = cache[distr];
    if (b.empty()) {
        const char *names[3] = {"beckmann", "ggx", "phong"};
        fs::path fn = Thread::getThread()->getFileResolver()->resolve(
            formatString("data/microfacet/%s.dat", names[distr]));
        std::ifstream is(fn.string().c_str(), std::ios::binary);
        b.assign(std::istreambuf_iterator<char>(is), std::istreambuf_iterator<char>());
        if (b.empty()) SLog(EError, "gpupath: could not read %s", fn.string().c_str());
    }
    return b;
}

} // namespace

class GPUIntegrator : public MonteCarloIntegrator {
public:
    GPUIntegrator(const Properties &props) : MonteCarloIntegrator(props), m_props(props) {
        /* "devices": comma-separated HIP device indices (default: current device) */
        std::istringstream is(props.getString("devices", "-1"));
        for (std::string tok; std::getline(is, tok, ',');)
            if (!tok.empty()) m_devices.push_back(atoi(tok.c_str()));
#if GPU_INTEGRATOR == 2
        /* direct.cpp:55-66 */
        const int shadingSamples = props.getSize("shadingSamples", 1);
        m_emitterSamples = props.getSize("emitterSamples", shadingSamples);
        m_bsdfSamples = props.getSize("bsdfSamples", shadingSamples);
        if (m_emitterSamples + m_bsdfSamples == 0)
            Log(EError, "Must have at least 1 BSDF or emitter sample!");
#endif
        /* the reference's CPU integrator behind Li() */
        Properties cpuProps(props);
        cpuProps.setPluginName(cpuPluginName());
        cpuProps.removeProperty("devices");
        m_cpu = static_cast<SamplingIntegrator *>(PluginManager::getInstance()->
            createObject(MTS_CLASS(Integrator), cpuProps));
        m_cpu->configure();
    }

    GPUIntegrator(Stream *stream, InstanceManager *manager)
        : MonteCarloIntegrator(stream, manager) {
        Log(EError, "gpupath renders on a local GPU; network rendering is not supported");
    }

    ~GPUIntegrator() {
        if (m_group) mtsgpu_group_destroy(m_group);
    }

    /* per-ray queries: the reference's own integrator */
    Spectrum Li(const RayDifferential &r, RadianceQueryRecord &rRec) const {
        return m_cpu->Li(r, rRec);
    }

    bool preprocess(const Scene *scene, RenderQueue *queue, const RenderJob *job,
                    int sceneResID, int sensorResID, int samplerResID) {
        MonteCarloIntegrator::preprocess(scene, queue, job, sceneResID, sensorResID, samplerResID);
        return m_cpu->preprocess(scene, queue, job, sceneResID, sensorResID, samplerResID);
    }

    void configureSampler(const Scene *scene, Sampler *sampler) {
        m_cpu->configureSampler(scene, sampler);      /* direct.cpp's request2DArray calls, if any */
    }

    bool render(Scene *scene, RenderQueue *queue, const RenderJob *job,
                int sceneResID, int sensorResID, int samplerResID) {
        ref<Sensor> sensor = scene->getSensor();
        ref<Film> film = sensor->getFilm();
        const Sampler *sampler = scene->getSampler();
        const std::string smpName = sampler->getClass()->getName();
        if (smpName != "SobolSampler" && smpName != "IndependentSampler")
            Log(EError, "%s supports the 'sobol' and 'independent' samplers", getClass()->getName().c_str());
        /* The 'perspective' plugin registers the concrete class PerspectiveCameraImpl
           (perspective.cpp:474) under the abstract PerspectiveCamera (sensor.cpp:319);
           'perspective_rdist' (PerspectiveCameraRDist, perspective_rdist.cpp:556) derives
           from it too but adds lens distortion, which the library does not model. */
        if (!sensor->getClass()->derivesFrom(MTS_CLASS(PerspectiveCamera))
            || sensor->getClass()->getName() != "PerspectiveCameraImpl")
            Log(EError, "only the 'perspective' sensor is supported (got %s)",
                sensor->getClass()->getName().c_str());
#if GPU_INTEGRATOR == 1
        if (sensor->getMedium())
            Log(EError, "gpuvolpath: participating media are not supported");
#endif
        m_cancelled = 0;

        std::vector<mtsgpu_mesh_desc> meshes;
        std::vector<const Emitter *> emitterObjs;
        m_bsdfs.clear(); m_bsdfObjs.clear(); m_keep.clear();
        m_sceneFile = scene->getSourceFile();    /* nested / textured BSDFs are read from it by id */
        std::vector<mtsgpu_emitter_desc> emitters;
        for (size_t i = 0; i < scene->getEmitters().size(); ++i) {   /* scene order = emitter PDF order */
            const Emitter *e = scene->getEmitters()[i].get();
            mtsgpu_emitter_desc d;
            std::memset(&d, 0, sizeof d);
            const Properties &p = e->getProperties();
            d.sampling_weight = (float) p.getFloat("samplingWeight", 1.0f);
            const std::string cls = e->getClass()->getName();
            if (cls == "EnvironmentMap") {
                /* the source image as EnvironmentMap's ctor loads it (envmap.cpp:117-160) */
                fs::path fn = Thread::getThread()->getFileResolver()->resolve(p.getString("filename"));
                ref<Bitmap> bmp = new Bitmap(Bitmap::EAuto, new FileStream(fn, FileStream::EReadOnly));
                if (p.getFloat("gamma", 0) != 0) bmp->setGamma(p.getFloat("gamma"));
                bmp = bmp->convert(Bitmap::ERGB, Bitmap::EFloat32, 1.0f, 1.0f, Spectrum::EIlluminant);
                d.type = MTSGPU_EMITTER_ENVMAP;
                d.env_rgb = bmp->getFloat32Data();
                d.env_width = (uint32_t) bmp->getWidth(); d.env_height = (uint32_t) bmp->getHeight();
                d.env_scale = (float) p.getFloat("scale", 1.0f);
                const Transform t = p.getTransform("toWorld", Transform());
                copyMatrix(t.getMatrix(), d.env_to_world);
                copyMatrix(t.getInverseMatrix(), d.env_to_world_inv);
                m_keep.push_back(bmp);
            } else if (cls == "ConstantBackgroundEmitter") {          /* constant.cpp */
                d.type = MTSGPU_EMITTER_CONSTANT;
                toRGB(p.getSpectrum("radiance", Spectrum::getD65()), d.radiance);
            } else if (cls == "AreaLight") {                          /* area.cpp */
                d.type = MTSGPU_EMITTER_AREA;
                toRGB(p.getSpectrum("radiance", Spectrum::getD65()), d.radiance);
            } else {
                Log(EError, "emitter \"%s\" is not supported", cls.c_str());
            }
            emitters.push_back(d);
            emitterObjs.push_back(e);
        }
        const ref_vector<Shape> &shapes = scene->getShapes();    /* kd-tree primitive order */
        for (size_t i = 0; i < shapes.size(); ++i) {
            const Shape *shape = shapes[i].get();
            const std::string cls = shape->getClass()->getName();
            mtsgpu_mesh_desc md;
            std::memset(&md, 0, sizeof md);
            md.bsdf = bsdfIndex(shape->getBSDF(), shape);
            md.emitter = shape->isEmitter() ? indexOf(emitterObjs, (const Emitter *) shape->getEmitter()) : -1;
            if (shape->hasMedium() || shape->isMediumTransition())
                Log(EError, "participating media are not supported");
            if (cls == "Rectangle" || cls == "Disk" || cls == "Sphere") {   /* analytic primitives */
                const Properties &p = shape->getProperties();
                md.shape_type = cls == "Rectangle" ? MTSGPU_SHAPE_RECTANGLE
                              : cls == "Disk" ? MTSGPU_SHAPE_DISK : MTSGPU_SHAPE_SPHERE;
                md.has_to_world = p.hasProperty("toWorld");
                const Transform t = p.getTransform("toWorld", Transform());   /* as the ctor reads it */
                copyMatrix(t.getMatrix(), md.to_world);
                copyMatrix(t.getInverseMatrix(), md.to_world_inv);
                const Point c = p.getPoint("center", Point(0.0f));
                md.center[0] = (float) c.x; md.center[1] = (float) c.y; md.center[2] = (float) c.z;
                md.radius = (float) p.getFloat("radius", 1.0f);
                md.flip_normals = p.getBoolean("flipNormals", false);
            } else if (shape->getClass()->derivesFrom(MTS_CLASS(TriMesh))) {
                const TriMesh *m = static_cast<const TriMesh *>(shape);   /* world space after configure() */
                md.shape_type = MTSGPU_SHAPE_TRIMESH;
                md.positions = (const float *) m->getVertexPositions();
                md.normals = m->hasVertexNormals() ? (const float *) m->getVertexNormals() : NULL;
                md.texcoords = m->hasVertexTexcoords() ? (const float *) m->getVertexTexcoords() : NULL;
                md.indices = (const uint32_t *) m->getTriangles();
                md.num_vertices = (uint32_t) m->getVertexCount();
                md.num_triangles = (uint32_t) m->getTriangleCount();
                md.face_normals = !m->hasVertexNormals();
            } else {
                Log(EError, "shape \"%s\" is not supported", cls.c_str());
            }
            meshes.push_back(md);
        }

        mtsgpu_scene_desc sd;
        std::memset(&sd, 0, sizeof sd);
        sd.meshes = meshes.data(); sd.num_meshes = (uint32_t) meshes.size();
        sd.bsdfs = m_bsdfs.data(); sd.num_bsdfs = (uint32_t) m_bsdfs.size();
        sd.emitters = emitters.data(); sd.num_emitters = (uint32_t) emitters.size();
        /* perspective.cpp: the derived x field of view, clip planes, camera-to-world */
        const PerspectiveCamera *cam = static_cast<const PerspectiveCamera *>(sensor.get());
        sd.sensor.fov = (float) cam->getXFov();
        sd.sensor.fov_axis = MTSGPU_FOV_X;
        sd.sensor.near_clip = (float) cam->getNearClip();
        sd.sensor.far_clip = (float) cam->getFarClip();
        copyMatrix(sensor->getWorldTransform()->eval(0).getMatrix(), sd.sensor.to_world);
        sd.sensor.film_width = (uint32_t) film->getSize().x;
        sd.sensor.film_height = (uint32_t) film->getSize().y;

        mtsgpu_render_params rp;
        std::memset(&rp, 0, sizeof rp);
        rp.spp = (uint32_t) sampler->getSampleCount();
        rp.scramble = (uint64_t) sampler->getProperties().getLong("scramble", 0);
        rp.sampler = smpName == "SobolSampler" ? MTSGPU_SAMPLER_SOBOL : MTSGPU_SAMPLER_INDEPENDENT;
#if GPU_INTEGRATOR == 2
        rp.integrator = MTSGPU_INTEGRATOR_DIRECT;
        rp.emitter_samples = (uint32_t) m_emitterSamples;
        rp.bsdf_samples = (uint32_t) m_bsdfSamples;
        rp.max_depth = 1; rp.rr_depth = 1;
#else
        rp.integrator = GPU_INTEGRATOR == 1 ? MTSGPU_INTEGRATOR_VOLPATH : MTSGPU_INTEGRATOR_PATH;
        rp.max_depth = m_maxDepth; rp.rr_depth = m_rrDepth;
#endif
        rp.strict_normals = m_strictNormals; rp.hide_emitters = m_hideEmitters;
        rp.has_alpha = film->hasAlpha();
        const ReconstructionFilter *rf = film->getReconstructionFilter();
        const std::string rfName = rf->getClass()->getName();
        if (rfName == "BoxFilter") {
            rp.rfilter = MTSGPU_RFILTER_BOX; rp.rfilter_param = (float) rf->getRadius();
        } else if (rfName == "GaussianFilter") {
            rp.rfilter = MTSGPU_RFILTER_GAUSSIAN;
            rp.rfilter_param = (float) rf->getProperties().getFloat("stddev", 0.5f);
        } else {
            Log(EError, "reconstruction filter \"%s\" is not supported (box, gaussian)", rfName.c_str());
        }
        rp.x0 = (uint32_t) film->getCropOffset().x; rp.y0 = (uint32_t) film->getCropOffset().y;
        rp.width = (uint32_t) film->getCropSize().x; rp.height = (uint32_t) film->getCropSize().y;
        rp.row_block = 8;                                /* (the group deals 8x8 tiles itself) */
        rp.cancel = &m_cancelled;

        if (!m_group) {
            std::vector<int> devs(m_devices.empty() ? std::vector<int>(1, -1) : m_devices);
            if (mtsgpu_group_create(devs.data(), (int) devs.size(), &m_group) != MTSGPU_OK)
                Log(EError, "%s: %s", getClass()->getName().c_str(), mtsgpu_group_last_error(NULL));
        }
        if (mtsgpu_group_upload_scene(m_group, &sd) != MTSGPU_OK)    /* configure() errors, as the reference words them */
            Log(EError, "%s", mtsgpu_group_last_error(m_group));

        const int b = mtsgpu_film_border(rp.rfilter, rp.rfilter_param);
        ref<ImageBlock> block = new ImageBlock(Bitmap::ESpectrumAlphaWeight, film->getSize(), rf);
        SAssert(block->getBorderSize() == b);
        const Vector2i full = block->getBitmap()->getSize();         /* (W+2b) x (H+2b) */
        std::vector<float> rgbaw((size_t) full.x * full.y * 5);
        mtsgpu_stats st;
        const int rc = mtsgpu_group_render(m_group, &rp, rgbaw.data(), &st);
        if (rc == MTSGPU_ECANCEL) return false;
        if (rc != MTSGPU_OK) Log(EError, "%s", mtsgpu_group_last_error(m_group));
        /* ImageBlock storage: ESpectrumAlphaWeight = SPECTRUM_SAMPLES + 2 Floats per pixel */
        Float *dst = block->getBitmap()->getFloatData();
        for (size_t i = 0; i < (size_t) full.x * full.y; ++i) {
            Spectrum s;
            s.fromLinearRGB(rgbaw[5 * i], rgbaw[5 * i + 1], rgbaw[5 * i + 2]);
            for (int c = 0; c < SPECTRUM_SAMPLES; ++c) dst[c] = s[c];
            dst[SPECTRUM_SAMPLES] = rgbaw[5 * i + 3];
            dst[SPECTRUM_SAMPLES + 1] = rgbaw[5 * i + 4];
            dst += SPECTRUM_SAMPLES + 2;
        }
        block->setOffset(Point2i(0, 0));
        film->put(block);                                 /* renderproc.cpp:142-149 */
        queue->signalRefresh(job);
        Log(EInfo, "%s: %llu samples, %llu rays, %llu shadow rays, %.1f ms on %d GPU(s)",
            getClass()->getName().c_str(), (unsigned long long) st.samples, (unsigned long long) st.rays,
            (unsigned long long) st.shadow_rays, st.kernel_ms, mtsgpu_group_size(m_group));
        return true;
    }

    void cancel() { m_cancelled = 1; }

    std::string toString() const {
        std::ostringstream oss;
        oss << getClass()->getName() << "[devices = " << m_props.getString("devices", "-1")
            << ", cpu = " << m_cpu->toString() << "]";
        return oss.str();
    }

    MTS_DECLARE_CLASS()
private:
    /* Does the BSDF give the same diffuse reflectance and roughness at every
       probed surface position (gpupath_probe_uv)?  Only for BSDFs the scene
       file does not hold (see bsdfIndex): a probe cannot prove a parameter
       constant, it can only catch a textured one. */
    static bool isConstant(const BSDF *bsdf) {
        std::vector<Intersection> its;
        const std::vector<std::pair<float, float> > uv = gpupath_probe_uv();
        for (size_t k = 0; k < uv.size(); ++k) {
            Intersection a;
            a.uv = Point2(uv[k].first, uv[k].second);
            a.p = Point(a.uv.x, a.uv.y, (Float) (k & 1));
            its.push_back(a);
        }
        const Spectrum r0 = bsdf->getDiffuseReflectance(its[0]);
        for (size_t k = 1; k < its.size(); ++k) {
            if (bsdf->getDiffuseReflectance(its[k]) != r0) return false;
            for (int c = 0; c < bsdf->getComponentCount(); ++c)
                if (bsdf->getRoughness(its[k], c) != bsdf->getRoughness(its[0], c)) return false;
        }
        return true;
    }

    /* Append a BSDF descriptor (de-duplicated by pointer); NULL -> -1 (the
       library applies Shape::configure's default diffuse, shape.cpp:48-70).
       The plugins keep textures and nested BSDFs as private children, out of
       reach of a plugin shim, so the scene file is the authority: every BSDF
       the file holds -- by its own id, or inline in a shape with an id -- is
       read back from it (mtsgpu_xml_bsdf_ex, Scene::getSourceFile) and
       converted from the rebuilt element tree.  Only a BSDF the file does not
       hold (a scene built in code, an inline BSDF of a shape without id) is
       converted from its Properties, and only when it is not twosided and the
       probe finds no varying parameter. */
    int bsdfIndex(const BSDF *bsdf, const Shape *shape) {
        if (!bsdf) return -1;
        const int have = indexOf(m_bsdfObjs, bsdf);
        if (have >= 0) return have;
        const std::string where = formatString("(the BSDF of shape \"%s\", id \"%s\")",
                                               shape->getName().c_str(), shape->getID().c_str());
        if (!m_sceneFile.empty()) {
            int idx = xmlBsdf(bsdf, bsdf->getID(), MTSGPU_XML_BY_ID, where);
            /* the meshes of a compound shape (OBJ, serialized) carry no <shape> id: TriMesh(name, ...)
               is built on empty Properties (trimesh.cpp:43), so its id is "unnamed" */
            if (idx == -2 && shape->getID() != "unnamed") idx = xmlBsdf(bsdf, shape->getID(), MTSGPU_XML_BY_SHAPE, where);
            if (idx >= 0) return idx;
        }
        const Properties &p = bsdf->getProperties();
        const std::string hint = shape->getID() == "unnamed"
            ? "a mesh of a compound shape (OBJ / serialized file) does not carry its <shape>'s id: give the BSDF "
              "itself an id (<bsdf id=...>, or a <ref> to one) in " : "give the BSDF (or its shape) an id in ";
        if (p.getPluginName() == "twosided")
            Log(EError, "twosided BSDF \"%s\" %s: its nested BSDFs are read from the scene file, which does not "
                "hold it; %s%s", bsdf->getID().c_str(), where.c_str(), hint.c_str(),
                m_sceneFile.empty() ? "a scene file" : m_sceneFile.string().c_str());
        if (!isConstant(bsdf))
            Log(EError, "BSDF \"%s\" %s has a textured parameter, and textures are read from the scene file, which "
                "does not hold it; %s%s", bsdf->getID().c_str(), where.c_str(), hint.c_str(),
                m_sceneFile.empty() ? "a scene file" : m_sceneFile.string().c_str());
        return appendDesc(p, bsdf, NULL);
    }

    /* The loader's parameters ($name substitutions): the integrator's
       'parameters' property ("name=value;name=value") if set, else the
       `mitsuba -D name=value` arguments of this process (mitsuba.cpp:168-173).
       They take precedence over the file's <default>s, as in the loader.
       Returns false when they cannot be known: no 'parameters' property, and this
       process is not the mitsuba command-line renderer (mtssrv, mtsgui, Python). */
    bool loaderParameters(std::vector<std::string> &names, std::vector<std::string> &values) const {
        std::string cmdline, bad;
        if (!m_props.hasProperty("parameters")) {
            std::ifstream is("/proc/self/cmdline", std::ios::binary);
            cmdline.assign(std::istreambuf_iterator<char>(is), std::istreambuf_iterator<char>());
        }
        bool known = true;
        if (!gpupath_loader_params(m_props.hasProperty("parameters"), m_props.getString("parameters", ""), cmdline,
                                   names, values, bad, &known))
            Log(EError, "Invalid parameter specification \"%s\"", bad.c_str());
        return known;
    }

    /* The file's tree for `id` -> descriptors; -2 when the file does not hold it */
    int xmlBsdf(const BSDF *bsdf, const std::string &id, int lookup, const std::string &where) {
        std::vector<std::string> pn, pv;
        const bool paramsKnown = loaderParameters(pn, pv);
        std::vector<const char *> pnc, pvc;
        for (size_t i = 0; i < pn.size(); ++i) { pnc.push_back(pn[i].c_str()); pvc.push_back(pv[i].c_str()); }
        std::vector<mtsgpu_xml_node> nodes(64);
        std::vector<mtsgpu_xml_prop> props(1024);
        int nn = 0, np = 0;
        char err[512] = "";
        const std::string file = m_sceneFile.string();
        int rc = mtsgpu_xml_bsdf_ex(file.c_str(), id.c_str(), lookup, pnc.data(), pvc.data(), (int32_t) pn.size(),
                                    nodes.data(), (int) nodes.size(), props.data(), (int) props.size(), &nn, &np,
                                    err, sizeof err);
        if (rc == MTSGPU_ENOMEM) {
            nodes.resize((size_t) nn); props.resize((size_t) np);
            rc = mtsgpu_xml_bsdf_ex(file.c_str(), id.c_str(), lookup, pnc.data(), pvc.data(), (int32_t) pn.size(),
                                    nodes.data(), nn, props.data(), np, &nn, &np, err, sizeof err);
        }
        if (rc == MTSGPU_ENOENT) return -2;
        if (rc != MTSGPU_OK)
            Log(EError, "BSDF \"%s\" %s, read from %s: %s", bsdf->getID().c_str(), where.c_str(), file.c_str(), err);
        nodes.resize((size_t) nn);
        props.resize((size_t) np);
        const Properties &have = bsdf->getProperties();
        /* by id: the element must describe this object.  An OBJ's .mtl materials are BSDFs
           whose id is the material name (obj.cpp:573) and which the file does not hold; an
           unrelated file element with that id differs from them in its plugin or in the set of
           its own properties (the loader sets exactly the file's properties on a BSDF it builds) */
        if (lookup == MTSGPU_XML_BY_ID) {
            bool same = std::string(nodes[0].plugin) == have.getPluginName();
            std::set<std::string> fileNames;
            for (int i = nodes[0].first_prop; i < nodes[0].first_prop + nodes[0].num_props; ++i)
                fileNames.insert(props[i].name);
            const std::vector<std::string> haveNames = have.getPropertyNames();
            same = same && fileNames.size() == haveNames.size();
            for (size_t k = 0; same && k < haveNames.size(); ++k) same = fileNames.count(haveNames[k]) != 0;
            if (!same) return -2;
        }
        if (std::string(nodes[0].plugin) != have.getPluginName())
            Log(EError, "BSDF \"%s\" %s is a \"%s\" in the scene but a \"%s\" in %s", bsdf->getID().c_str(),
                where.c_str(), have.getPluginName().c_str(), nodes[0].plugin, file.c_str());
        for (size_t i = 0; i < props.size(); ++i)
            if (!paramsKnown && (props[i].flags & MTSGPU_XML_PROP_PARAM))
                Log(EError, "BSDF \"%s\" %s: %s uses $parameters (\"%s\"), and this process is not the mitsuba "
                    "renderer, whose -D arguments they would be: set the integrator's 'parameters' property to the "
                    "loader's name=value list", bsdf->getID().c_str(), where.c_str(), file.c_str(), props[i].name);
        /* The top BSDF's own properties are visible: a value the file's <default>
           supplied must be the one the loader used, or the loader had a parameter
           this shim was not given (nested elements could differ the same way). */
        Properties fromFile(nodes[0].plugin);
        for (int i = nodes[0].first_prop; i < nodes[0].first_prop + nodes[0].num_props; ++i) {
            if (props[i].flags & MTSGPU_XML_PROP_UNSUPPORTED) continue;   /* taken from `have` (xmlNode) */
            setProperty(fromFile, props[i]);
            const std::string name = props[i].name;
            if ((props[i].flags & MTSGPU_XML_PROP_DEFAULT) && have.hasProperty(name) &&
                have.getAsString(name) != fromFile.getAsString(name))
                Log(EError, "BSDF \"%s\" %s: property \"%s\" is %s in the scene but %s by the file's <default>: "
                    "the loader had parameters this integrator was not given (set its 'parameters' property to "
                    "the loader's name=value list)", bsdf->getID().c_str(), where.c_str(), name.c_str(),
                    have.getAsString(name).c_str(), fromFile.getAsString(name).c_str());
        }
        return xmlNode(nodes, props, 0, bsdf);
    }

    /* one node of the file's tree (and its subtree) -> descriptors */
    int xmlNode(const std::vector<mtsgpu_xml_node> &nodes, const std::vector<mtsgpu_xml_prop> &props, int k,
                const BSDF *obj) {
        Properties p(nodes[k].plugin);
        for (int i = nodes[k].first_prop; i < nodes[k].first_prop + nodes[k].num_props; ++i) {
            if (!(props[i].flags & MTSGPU_XML_PROP_UNSUPPORTED)) {
                setProperty(p, props[i]);
                continue;
            }
            /* <spectrum filename=...>, a sampled spectrum, <blackbody>: the loader's parsed value,
               which only the top BSDF's own Properties expose */
            const std::string name = props[i].name;
            if (k != 0 || !obj || !obj->getProperties().hasProperty(name))
                Log(EError, "<%s name=\"%s\" %s> in a nested element of BSDF \"%s\": this form is only supported "
                    "on the top BSDF (or give it as a value)", props[i].tag, props[i].name, props[i].value,
                    obj ? obj->getID().c_str() : nodes[0].id);
            p.copyAttribute(obj->getProperties(), name, name);
        }
        std::vector<std::pair<std::string, mtsgpu_texture_desc> > tex;
        std::vector<int> nested;
        for (int c = k + 1; c < (int) nodes.size(); ++c) {
            if (nodes[c].parent != k) continue;
            if (nodes[c].kind == MTSGPU_XML_TEXTURE) tex.push_back(std::make_pair(std::string(nodes[c].name),
                                                                                  textureDesc(nodes[c], props)));
            else nested.push_back(c);
        }
        if (p.getPluginName() == "twosided") {                   /* twosided.cpp:63-110, 193-205 */
            if (nested.empty()) Log(EError, "A nested one-sided material is required!");
            if (nested.size() > 2) Log(EError, "No more than two nested BRDFs can be added!");
            mtsgpu_bsdf_desc d;
            std::memset(&d, 0, sizeof d);
            d.type = MTSGPU_BSDF_TWOSIDED;
            d.nested[0] = d.nested[1] = -1;
            const int idx = (int) m_bsdfs.size();
            m_bsdfs.push_back(d);
            m_bsdfObjs.push_back(obj);
            for (size_t j = 0; j < nested.size(); ++j) {
                const int ni = xmlNode(nodes, props, nested[j], NULL);
                m_bsdfs[idx].nested[j] = ni;
            }
            return idx;
        }
        if (!nested.empty()) Log(EError, "%s: nested BSDFs are only supported inside twosided", nodes[k].plugin);
        return appendDesc(p, obj, &tex);
    }

    /* a property element of the file as the scene loader would set it (scenehandler.cpp) */
    static void setProperty(Properties &p, const mtsgpu_xml_prop &e) {
        const std::string tag = e.tag, name = e.name, v = e.value;
        std::vector<Float> f;
        {
            std::string t = v;
            for (size_t i = 0; i < t.size(); ++i) if (t[i] == ',') t[i] = ' ';
            std::istringstream is(t);
            for (Float x; is >> x;) f.push_back(x);
        }
        if (tag == "float") p.setFloat(name, f.empty() ? 0 : f[0]);
        else if (tag == "integer") p.setInteger(name, atoi(v.c_str()));
        else if (tag == "boolean") p.setBoolean(name, v == "true");
        else if (tag == "string") p.setString(name, v);
        else if (tag == "point" && f.size() == 3) p.setPoint(name, Point(f[0], f[1], f[2]));
        else if (tag == "vector" && f.size() == 3) p.setVector(name, Vector(f[0], f[1], f[2]));
        else if (tag == "rgb" || tag == "srgb") {
            Spectrum s;
            if (tag == "srgb" && !v.empty() && v[0] == '#') {
                const unsigned long c = strtoul(v.c_str() + 1, NULL, 16);
                s.fromSRGB(((c >> 16) & 0xff) / 255.0f, ((c >> 8) & 0xff) / 255.0f, (c & 0xff) / 255.0f);
            } else if (f.size() == 1 || f.size() == 3) {
                const Float r = f[0], g = f.size() == 3 ? f[1] : f[0], b = f.size() == 3 ? f[2] : f[0];
                if (tag == "srgb") s.fromSRGB(r, g, b); else s.fromLinearRGB(r, g, b);
            } else {
                SLog(EError, "could not parse <%s name=\"%s\" value=\"%s\">", e.tag, e.name, e.value);
            }
            p.setSpectrum(name, s);
        } else if (tag == "spectrum" && f.size() == 1 && v.find(':') == std::string::npos) {
            p.setSpectrum(name, Spectrum(f[0]));
        } else {
            SLog(EError, "<%s name=\"%s\" value=\"%s\"> in a nested or textured BSDF is not supported",
                 e.tag, e.name, e.value);
        }
    }

    /* checkerboard (textures/checkerboard.cpp) with Texture2D's uv transform (texture.cpp:81-95) */
    static mtsgpu_texture_desc textureDesc(const mtsgpu_xml_node &n, const std::vector<mtsgpu_xml_prop> &props) {
        if (std::string(n.plugin) != "checkerboard")
            SLog(EError, "texture \"%s\" is not supported (checkerboard)", n.plugin);
        Properties p(n.plugin);
        for (int i = n.first_prop; i < n.first_prop + n.num_props; ++i) setProperty(p, props[i]);
        mtsgpu_texture_desc t;
        std::memset(&t, 0, sizeof t);
        t.type = MTSGPU_TEX_CHECKERBOARD;
        toRGB(p.getSpectrum("color0", Spectrum(.4f)), t.color0);
        toRGB(p.getSpectrum("color1", Spectrum(.2f)), t.color1);
        t.uoffset = (float) p.getFloat("uoffset", 0.0f);
        t.voffset = (float) p.getFloat("voffset", 0.0f);
        const Float uvscale = p.getFloat("uvscale", 1.0f);
        t.uscale = (float) p.getFloat("uscale", uvscale);
        t.vscale = (float) p.getFloat("vscale", uvscale);
        return t;
    }

    /* a descriptor from a BSDF's Properties; `tex`: its texture children (name -> texture) */
    int appendDesc(const Properties &p, const BSDF *bsdf,
                   const std::vector<std::pair<std::string, mtsgpu_texture_desc> > *tex) {
        const std::string name = p.getPluginName();
        mtsgpu_bsdf_desc d;
        std::memset(&d, 0, sizeof d);
        d.nested[0] = d.nested[1] = -1;
        d.type = name == "diffuse" ? MTSGPU_BSDF_DIFFUSE : name == "roughconductor" ? MTSGPU_BSDF_ROUGHCONDUCTOR
               : name == "roughdielectric" ? MTSGPU_BSDF_ROUGHDIELECTRIC : name == "roughplastic" ? MTSGPU_BSDF_ROUGHPLASTIC
               : name == "conductor" ? MTSGPU_BSDF_CONDUCTOR : name == "dielectric" ? MTSGPU_BSDF_DIELECTRIC
               : name == "plastic" ? MTSGPU_BSDF_PLASTIC : -1;
        if (d.type < 0) Log(EError, "BSDF \"%s\" is not supported", name.c_str());
        d.distribution = distribution(p);
        d.sample_visible = p.getBoolean("sampleVisible", true);
        d.ensure_energy_conservation = p.getBoolean("ensureEnergyConservation", true);
        const Float alpha = p.getFloat("alpha", 0.1f);
        d.alpha_u = (float) p.getFloat("alphaU", alpha);
        d.alpha_v = (float) p.getFloat("alphaV", alpha);
        toRGB(p.getSpectrum("reflectance", Spectrum(.5f)), d.reflectance);
        toRGB(p.getSpectrum("specularReflectance", Spectrum(1.0f)), d.specular_reflectance);
        toRGB(p.getSpectrum("specularTransmittance", Spectrum(1.0f)), d.specular_transmittance);
        toRGB(p.getSpectrum("diffuseReflectance", Spectrum(.5f)), d.diffuse_reflectance);
        d.nonlinear = p.getBoolean("nonlinear", false);
        if (d.type == MTSGPU_BSDF_ROUGHCONDUCTOR || d.type == MTSGPU_BSDF_CONDUCTOR) {
            /* roughconductor.cpp:169-190 / conductor.cpp: 'material' spectra -> RGB by the
               reference's own InterpolatedSpectrum; the library divides by extEta */
            ref<FileResolver> fr = Thread::getThread()->getFileResolver();
            const std::string mat = p.getString("material", "Cu");
            Spectrum intEta(0.0f), intK(1.0f);
            std::string lower = mat;
            for (size_t i = 0; i < lower.size(); ++i) lower[i] = (char) tolower(lower[i]);
            if (lower != "none") {
                intEta.fromContinuousSpectrum(InterpolatedSpectrum(fr->resolve("data/ior/" + mat + ".eta.spd")));
                intK.fromContinuousSpectrum(InterpolatedSpectrum(fr->resolve("data/ior/" + mat + ".k.spd")));
            }
            toRGB(p.getSpectrum("eta", intEta), d.eta);
            toRGB(p.getSpectrum("k", intK), d.k);
            d.ext_eta = (float) lookupIOR(p, "extEta", "air");
        }
        const bool plastic = d.type == MTSGPU_BSDF_ROUGHPLASTIC || d.type == MTSGPU_BSDF_PLASTIC;
        d.int_ior = (float) lookupIOR(p, "intIOR", plastic ? "polypropylene" : "bk7");
        d.ext_ior = (float) lookupIOR(p, "extIOR", "air");
        if (d.type == MTSGPU_BSDF_ROUGHPLASTIC) {
            const std::vector<char> &b = rtransBytes(d.distribution);
            d.rtrans_data = b.data();
            d.rtrans_bytes = b.size();
        }
        for (size_t i = 0; tex && i < tex->size(); ++i) {      /* BSDF::addChild of a texture */
            const std::string &pn = (*tex)[i].first;
            if (pn == "alpha" && (d.type == MTSGPU_BSDF_ROUGHCONDUCTOR || d.type == MTSGPU_BSDF_ROUGHDIELECTRIC
                                  || d.type == MTSGPU_BSDF_ROUGHPLASTIC))
                d.alpha_tex = (*tex)[i].second;
            else if ((pn == "reflectance" && d.type == MTSGPU_BSDF_DIFFUSE) ||
                     (pn == "diffuseReflectance" && (d.type == MTSGPU_BSDF_ROUGHPLASTIC || d.type == MTSGPU_BSDF_PLASTIC)))
                d.reflectance_tex = (*tex)[i].second;
            else
                Log(EError, "%s: unsupported texture parameter \"%s\"", name.c_str(), pn.c_str());
        }
        m_bsdfs.push_back(d);
        m_bsdfObjs.push_back(bsdf);
        return (int) m_bsdfs.size() - 1;
    }

    Properties m_props;
    std::vector<int> m_devices;
    ref<SamplingIntegrator> m_cpu;
    mtsgpu_group *m_group = NULL;
    volatile int32_t m_cancelled = 0;
    std::vector<mtsgpu_bsdf_desc> m_bsdfs;
    std::vector<const BSDF *> m_bsdfObjs;          /* parallel to m_bsdfs (NULL: a nested BSDF) */
    fs::path m_sceneFile;
    ref_vector<Bitmap> m_keep;
#if GPU_INTEGRATOR == 2
    int m_emitterSamples = 1, m_bsdfSamples = 1;
#endif
};

MTS_IMPLEMENT_CLASS_S(GPUIntegrator, false, MonteCarloIntegrator)
MTS_EXPORT_PLUGIN(GPUIntegrator, "MI355X integrator (libmtsgpu): path / volpath / direct on the GPU");
MTS_NAMESPACE_END
