// Host-parser robustness check under AddressSanitizer + UndefinedBehaviorSanitizer (CPU only).
//
// Built by `make sanitize` from the host sources themselves with -fsanitize=address,undefined
// (pathtracercuda_amd/lib/host_sanitize_check) and run by tests/test_host.py.  The inputs are the
// untrusted files the reference reads (SceneLoader.cpp:199-219 scene JSON, Pathtracer.cpp:245-251
// textures): every committed scene and texture, then deterministic mutations of each -- truncations
// at every length up to 4 KiB (and a sample beyond), byte flips, and structural edits -- parsed
// with the same entry points the library uses.  The scenes that parse are also turned into
// CpuHittables and a BVH (the setScene path without a GPU) and the images written back out.
// Exit status 0 and no sanitizer report = pass.  No GPU call is made.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "pathtracer_amd.hpp"

static std::string readAll(const std::string& p)
{
    std::ifstream f(p, std::ios::binary);
    std::stringstream ss;
    ss << f.rdbuf();
    return ss.str();
}

static void writeAll(const std::string& p, const std::string& d)
{
    std::ofstream f(p, std::ios::binary | std::ios::trunc);
    f.write(d.data(), (std::streamsize)d.size());
}

static uint64_t g_state = 0x9E3779B97F4A7C15ull;
static uint32_t rnd()
{
    g_state ^= g_state << 13;
    g_state ^= g_state >> 7;
    g_state ^= g_state << 17;
    return (uint32_t)g_state;
}

static uint32_t noTextures(void*, const std::string&) { return 0; }

static size_t g_parsed = 0, g_rejected = 0;

static void tryScene(const std::string& path)
{
    ptamd::SceneDesc desc;
    std::string err;
    if (!ptamd::parseSceneFile(path, desc, err, noTextures, nullptr)) {
        ++g_rejected;
        return;
    }
    ++g_parsed;
    if (!desc.objects.empty() && desc.objects.size() <= 200000) {
        BVH bvh;
        bvh.build(desc.objects.size(), desc.objects.data(), 4);
        if (!bvh.validate()) {
            fprintf(stderr, "BVH validation failed for %s\n", path.c_str());
            exit(3);
        }
    }
}

static void tryImage(const std::string& path, const std::string& outDir)
{
    std::vector<float> rgba;
    uint32_t w = 0, h = 0;
    std::string err;
    if (!ptamd::loadImageRGBA32F(path, rgba, w, h, err)) {
        ++g_rejected;
        return;
    }
    ++g_parsed;
    if ((size_t)w * h * 4 != rgba.size()) {
        fprintf(stderr, "image size mismatch for %s\n", path.c_str());
        exit(4);
    }
    if ((size_t)w * h <= (1u << 22)) {
        std::vector<uint8_t> ldr(rgba.size());
        for (size_t i = 0; i < rgba.size(); ++i) ldr[i] = (uint8_t)(rgba[i] > 1.0f ? 255 : rgba[i] < 0.0f ? 0 : rgba[i] * 255.0f);
        ptamd::writePNG(outDir + "/rt.png", w, h, ldr.data(), true);
        ptamd::writeHDR(outDir + "/rt.hdr", w, h, rgba.data(), true);
    }
}

int main(int argc, char** argv)
{
    if (argc < 3) {
        fprintf(stderr, "usage: host_sanitize_check <tmpdir> <scene-or-image>...\n");
        return 2;
    }
    const std::string tmp = argv[1];
    for (int a = 2; a < argc; ++a) {
        const std::string path = argv[a];
        const std::string data = readAll(path);
        const bool image = path.size() > 4 && (path.substr(path.size() - 4) == ".png" || path.substr(path.size() - 4) == ".hdr");
        auto run = [&](const std::string& bytes) {
            const std::string p = tmp + (image ? (path.substr(path.size() - 4)) : std::string(".json"));
            const std::string q = tmp + "/case" + (image ? path.substr(path.size() - 4) : std::string(".json"));
            (void)p;
            writeAll(q, bytes);
            if (image) tryImage(q, tmp);
            else tryScene(q);
        };
        run(data);                                                      // the file itself
        const size_t dense = std::min<size_t>(data.size(), 4096);
        for (size_t n = 0; n < dense; n += image ? 7 : 3) run(data.substr(0, n));   // truncations
        for (int k = 0; k < 64 && data.size() > dense; ++k) run(data.substr(0, dense + rnd() % (data.size() - dense)));
        for (int k = 0; k < 400 && !data.empty(); ++k) {                // byte flips / overwrites
            std::string m = data;
            const int edits = 1 + (int)(rnd() % 4);
            for (int e = 0; e < edits; ++e) {
                const size_t at = (k < 200 && data.size() > 512) ? rnd() % 512 : rnd() % data.size();
                m[at] = (char)(rnd() & 0xff);
            }
            run(m);
        }
        if (!image) {                                                   // structural edits
            const char* junk[] = {"[", "]", "{", "}", ",", ":", "\"", "1e999", "-0", "null", "\"type\":", "9999999999999999999999"};
            for (int k = 0; k < 300; ++k) {
                std::string m = data;
                m.insert(rnd() % (m.size() + 1), junk[rnd() % (sizeof(junk) / sizeof(junk[0]))]);
                run(m);
            }
        }
    }
    printf("host_sanitize_check: %zu inputs parsed, %zu rejected, no sanitizer report\n", g_parsed, g_rejected);
    return 0;
}
