/*
 * gpupath_util.h -- the parts of the plugin shim (gpupath.cpp) that need no
 * Mitsuba header, so that tests/test_shim_util.py can compile and run them
 * here (the shim itself needs boost, which this image lacks).
 *
 *   gpupath_probe_uv        the surface positions at which the shim evaluates
 *                           a BSDF the scene file does not hold, to refuse a
 *                           textured one instead of rendering its defaults;
 *   gpupath_loader_params   the loader's $parameters: the integrator's
 *                           'parameters' property, else -- in the mitsuba
 *                           command-line renderer only -- the process's
 *                           `mitsuba -D name=value` arguments
 *                           (src/mitsuba/mitsuba.cpp:168-173, getopt syntax:
 *                           "-D", "a=b" or "-Da=b"; tokenize on '=').
 */
#ifndef GPUPATH_UTIL_H
#define GPUPATH_UTIL_H

#include <string>
#include <utility>
#include <vector>

/* Cell centres of a 16 x 16 grid over [0,1)^2, then an 8 x 8 grid of steps
   of 2 over [-8,8)^2 (off the cell corners).  Under Texture2D's uv transform
   (texture.cpp:81-95) and checkerboard's cells of 1/2 (checkerboard.cpp:66-74)
   the two grids see both colours of every checkerboard with uscale, vscale in
   [1/8 .. 8] at the offsets tests/test_shim_util.py sweeps.
   The round-4 probe, (0.173, 0.291) and (0.618, 0.854), fell in cells (0,0) and
   (1,1) of the default checkerboard: both color0. */
inline std::vector<std::pair<float, float> > gpupath_probe_uv() {
    std::vector<std::pair<float, float> > uv;
    for (int i = 0; i < 16; ++i)
        for (int j = 0; j < 16; ++j)
            uv.push_back(std::make_pair((i + 0.5f) / 16, (j + 0.5f) / 16));
    for (int i = 0; i < 8; ++i)
        for (int j = 0; j < 8; ++j)
            uv.push_back(std::make_pair(-8.0f + 2 * i + 0.37f, -8.0f + 2 * j + 0.61f));
    return uv;
}

/* mitsuba.cpp's tokenize(optarg, "="): the pieces between '=' characters, empty
   ones dropped ("a==b" and "=a=b" give a and b) */
inline std::vector<std::string> gpupath_tokenize_eq(const std::string &s) {
    std::vector<std::string> t;
    size_t b = 0;
    while (b <= s.size()) {
        size_t e = s.find('=', b);
        if (e == std::string::npos) e = s.size();
        if (e > b) t.push_back(s.substr(b, e - b));
        b = e + 1;
    }
    return t;
}

/* name=value pairs.  `property`: the 'parameters' property ("a=1;b=2"), used
   when `has_property`; otherwise `argv` (the NUL-separated /proc/self/cmdline),
   but only when argv[0] is the mitsuba command-line renderer: under mtssrv,
   mtsgui or the Python bindings the -D arguments belong to another program,
   and *known is set to false (no parameters are returned).  A pair is split as
   mitsuba.cpp:168-173 splits it (tokenize on '=', exactly two tokens); returns
   false (and the offending token in `bad`) for one the loader rejects with
   "Invalid parameter specification". */
inline bool gpupath_loader_params(bool has_property, const std::string &property, const std::string &cmdline,
                                  std::vector<std::string> &names, std::vector<std::string> &values,
                                  std::string &bad, bool *known = 0) {
    std::vector<std::string> pairs;
    if (known) *known = true;
    if (has_property) {
        size_t b = 0;
        while (b <= property.size()) {
            size_t e = property.find(';', b);
            if (e == std::string::npos) e = property.size();
            if (e > b) pairs.push_back(property.substr(b, e - b));
            b = e + 1;
        }
    } else {
        std::vector<std::string> argv;
        size_t b = 0;
        while (b < cmdline.size()) {
            size_t e = cmdline.find('\0', b);
            if (e == std::string::npos) e = cmdline.size();
            argv.push_back(cmdline.substr(b, e - b));
            b = e + 1;
        }
        const std::string exe = argv.empty() ? std::string() : argv[0].substr(argv[0].find_last_of('/') + 1);
        if (exe != "mitsuba") {
            if (known) *known = false;
            return true;
        }
        for (size_t i = 1; i < argv.size(); ++i) {
            if (argv[i] == "--") break;
            if (argv[i] == "-D" && i + 1 < argv.size()) pairs.push_back(argv[++i]);
            else if (argv[i].compare(0, 2, "-D") == 0 && argv[i].size() > 2) pairs.push_back(argv[i].substr(2));
        }
    }
    for (size_t i = 0; i < pairs.size(); ++i) {
        const std::vector<std::string> t = gpupath_tokenize_eq(pairs[i]);
        if (t.size() != 2) {
            bad = pairs[i];
            return false;
        }
        names.push_back(t[0]);
        values.push_back(t[1]);
    }
    return true;
}

#endif
