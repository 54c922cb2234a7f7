// Scene file loading (reference src/SceneLoader.cpp:124-348): JSON objects -> CpuHittable list,
// textures (memoised by path, loaded in order of first use, skybox after the objects), camera.
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <map>
#include <sstream>

#include "json_min.h"
#include "pathtracer_amd.hpp"

namespace ptamd {
namespace {

using json::Kind;
using json::Value;

bool getString(const Value& o, const char* key, std::string& out)
{
    const Value v = o.get(key);
    if (v.kind() == Kind::String) { out = std::string(v.str()); return true; }
    return false;
}

bool getFloat(const Value& o, const char* key, float& out)      // only JSON floats (is_number_float)
{
    const Value v = o.get(key);
    if (v.isFloat()) { out = (float)v.f(); return true; }
    return false;
}

bool getVec3(const Value& o, const char* key, vec3& out)
{
    const Value v = o.get(key);
    if (v.kind() == Kind::Array && v.size() == 3) {
        // get<float>() on a non-number throws in nlohmann; treat such a file as malformed here
        for (uint32_t k = 0; k < 3; ++k)
            if (!v.at(k).isNumber()) return false;
        out = vec3(v.at(0).asFloat(), v.at(1).asFloat(), v.at(2).asFloat());
        return true;
    }
    return false;
}

Value getObject(const Value& o, const char* key)
{
    const Value v = o.get(key);
    return v.kind() == Kind::Object ? v : Value();
}

} // namespace

bool parseSceneFile(const std::string& path, SceneDesc& out, std::string& error,
                    uint32_t (*textureLoader)(void* user, const std::string& path), void* user)
{
    std::ifstream file(path, std::ios::binary);
    if (!file.is_open()) {
        error = "Failed to open input file: " + path;
        return false;
    }
    std::string text;
    file.seekg(0, std::ios::end);
    const std::streamoff size = file.tellg();
    file.seekg(0, std::ios::beg);
    if (size > 0) {
        text.resize((size_t)size);
        file.read(&text[0], size);
        text.resize((size_t)file.gcount());
    }
    json::Document doc;
    if (!json::parse(text, doc, error)) return false;
    const Value root = json::root(doc);

    out = SceneDesc();
    std::map<std::string, uint32_t> handles;
    auto textureHandle = [&](const std::string& p) -> uint32_t {
        if (p.empty()) return 0;
        auto it = handles.find(p);
        if (it != handles.end()) return it->second;
        const uint32_t h = textureLoader ? textureLoader(user, p) : 0;
        handles[p] = h;
        if (h != 0) {
            if (out.texturePaths.size() < h) out.texturePaths.resize(h);
            out.texturePaths[h - 1] = p;
        }
        return h;
    };

    const Value objs = root.get("objects");
    if (objs.kind() == Kind::Array) {
        out.hasObjects = true;
        out.objects.reserve(objs.size());
        for (uint32_t oi = 0; oi < objs.size(); ++oi) {
            const Value o = objs.at(oi);
            HittableType htype = HittableType::SPHERE;
            vec3 position = 0.0f, rotation = 0.0f, scale = 1.0f;
            MaterialType mtype = MaterialType::LAMBERT;
            vec3 baseColor = 1.0f, emissive = 0.0f;
            float roughness = 0.5f, metalness = 0.0f;
            uint32_t tex = 0;
            std::string t;
            if (getString(o, "type", t)) {
                static const char* names[] = {"SPHERE", "CYLINDER", "DISK", "CONE", "PARABOLOID", "QUAD", "CUBE"};
                bool found = false;
                for (uint32_t k = 0; k < 7; ++k)
                    if (t == names[k]) { htype = (HittableType)k; found = true; }
                if (!found) { printf("Failed to parse object type: %s\n", t.c_str()); fflush(stdout); }
            }
            getVec3(o, "position", position);
            getVec3(o, "rotation", rotation);
            getVec3(o, "scale", scale);
            if (const Value m = getObject(o, "material"); m.valid()) {
                std::string mt;
                if (getString(m, "type", mt)) {
                    if (mt == "LAMBERT") mtype = MaterialType::LAMBERT;
                    else if (mt == "GGX") mtype = MaterialType::GGX;
                    else if (mt == "LAMBERT_GGX") mtype = MaterialType::LAMBERT_GGX;
                    else { printf("Failed to parse material type: %s\n", mt.c_str()); fflush(stdout); }
                }
                getVec3(m, "baseColor", baseColor);
                getVec3(m, "emissive", emissive);
                getFloat(m, "roughness", roughness);
                getFloat(m, "metalness", metalness);
                std::string tp;
                if (getString(m, "texture", tp)) tex = textureHandle(tp);
            }
            out.objects.push_back(CpuHittable(htype, position,
                                              vec3(radians(rotation.x), radians(rotation.y), radians(rotation.z)), scale,
                                              Material(mtype, baseColor, emissive, roughness, metalness, tex)));
        }
    }
    std::string sky;
    if (getString(root, "skybox", sky)) {
        out.hasSkybox = true;
        out.skyboxHandle = textureHandle(sky);
    }
    if (const Value c = getObject(root, "camera"); c.valid()) {
        getVec3(c, "position", out.cameraPosition);
        getVec3(c, "look_at", out.cameraLookAt);
        getFloat(c, "fovy", out.cameraFovyDegrees);
    }
    return true;
}

} // namespace ptamd

// Texture paths are resolved against the CWD as in the reference (SceneLoader.cpp:145); a path
// that does not exist there is retried relative to the scene file's directory (additive).
static std::string resolveTexturePath(const std::string& scenePath, const std::string& p)
{
    std::ifstream f(p, std::ios::binary);
    if (f.good()) return p;
    const size_t slash = scenePath.find_last_of('/');
    if (slash == std::string::npos) return p;
    const std::string alt = scenePath.substr(0, slash + 1) + p;
    std::ifstream g(alt, std::ios::binary);
    return g.good() ? alt : p;
}

struct LoadCtx {
    Pathtracer* pt;
    std::string scenePath;
};

static uint32_t loadTextureCb(void* user, const std::string& path)
{
    LoadCtx* c = (LoadCtx*)user;
    return c->pt->loadTexture(resolveTexturePath(c->scenePath, path).c_str());
}

Camera loadScene(Pathtracer& pathtracer, const Params& params)
{
    ptamd::SceneDesc desc;
    std::string error;
    LoadCtx ctx{&pathtracer, params.m_inputFilepath ? params.m_inputFilepath : ""};
    if (!ptamd::parseSceneFile(ctx.scenePath, desc, error, loadTextureCb, &ctx)) {
        printf("%s\n", error.c_str());
        exit(EXIT_FAILURE);
    }
    if (desc.hasObjects) pathtracer.setScene(desc.objects.size(), desc.objects.data());
    if (desc.hasSkybox) pathtracer.setSkyboxTextureHandle(desc.skyboxHandle);
    return Camera(desc.cameraPosition, desc.cameraLookAt, vec3(0.0f, 1.0f, 0.0f), ptamd::radians(desc.cameraFovyDegrees),
                  (float)params.m_width / params.m_height);
}
