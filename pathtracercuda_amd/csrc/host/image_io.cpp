// Image I/O for textures and output files, with stb_image / stb_image_write semantics for the
// formats the project uses (the reference vendors stb v2.26 / v1.15):
//   * Radiance .hdr read: RGBE -> float, f = ldexp(1, e - 136), alpha 1 (stb_image.h:7036-7061),
//     flat and new-style RLE scanlines;
//   * PNG read (8/16-bit gray, gray+alpha, RGB, RGBA, palette; non-interlaced) -> RGBA8, then
//     normalised c / 255 as a cudaReadModeNormalizedFloat texture reads it;
//   * PNG / HDR write of RGBA rows with optional vertical flip (main.cpp:184-197).
#include <zlib.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>

#include "pathtracer_amd.hpp"

namespace ptamd {
namespace {

bool readFile(const std::string& path, std::string& data)
{
    std::ifstream f(path, std::ios::binary);
    if (!f.is_open()) return false;
    std::stringstream ss;
    ss << f.rdbuf();
    data = ss.str();
    return true;
}

bool loadHDR(const std::string& data, std::vector<float>& rgba, uint32_t& w, uint32_t& h, std::string& err)
{
    size_t pos = 0;
    auto line = [&](std::string& out) -> bool {
        size_t e = data.find('\n', pos);
        if (e == std::string::npos) return false;
        out = data.substr(pos, e - pos);
        pos = e + 1;
        return true;
    };
    std::string s;
    if (!line(s) || (s != "#?RADIANCE" && s != "#?RGBE")) { err = "not a Radiance file"; return false; }
    bool fmtOk = false;
    while (true) {
        if (!line(s)) { err = "truncated header"; return false; }
        if (s.empty()) break;
        if (s == "FORMAT=32-bit_rle_rgbe") fmtOk = true;
    }
    if (!fmtOk) { err = "unsupported HDR format"; return false; }
    if (!line(s)) { err = "missing dimensions"; return false; }
    int hh = 0, ww = 0;
    if (sscanf(s.c_str(), "-Y %d +X %d", &hh, &ww) != 2 || hh <= 0 || ww <= 0 || hh > (1 << 24) || ww > (1 << 24)) {
        err = "unsupported HDR orientation/dimensions";
        return false;
    }
    w = (uint32_t)ww;
    h = (uint32_t)hh;
    std::vector<uint8_t> rgbe((size_t)w * h * 4);
    const uint8_t* d = (const uint8_t*)data.data();
    const size_t n = data.size();
    for (uint32_t j = 0; j < h; ++j) {
        uint8_t* row = &rgbe[(size_t)j * w * 4];
        if (w >= 8 && w < 32768 && pos + 4 <= n && d[pos] == 2 && d[pos + 1] == 2 && !(d[pos + 2] & 0x80)) {
            if (((uint32_t)d[pos + 2] << 8 | d[pos + 3]) != w) { err = "invalid RLE scanline width"; return false; }
            pos += 4;
            for (int k = 0; k < 4; ++k) {
                uint32_t i = 0;
                while (i < w) {
                    if (pos >= n) { err = "truncated RLE data"; return false; }
                    uint32_t count = d[pos++];
                    if (count > 128) {
                        count -= 128;
                        if (pos >= n || i + count > w) { err = "bad RLE run"; return false; }
                        const uint8_t v = d[pos++];
                        for (uint32_t c = 0; c < count; ++c) row[4 * (i + c) + k] = v;
                    } else {
                        if (count == 0 || pos + count > n || i + count > w) { err = "bad RLE dump"; return false; }
                        for (uint32_t c = 0; c < count; ++c) row[4 * (i + c) + k] = d[pos++];
                    }
                    i += count;
                }
            }
        } else {
            if (pos + 4 * (size_t)w > n) { err = "truncated HDR data"; return false; }
            memcpy(row, d + pos, 4 * (size_t)w);
            pos += 4 * (size_t)w;
        }
    }
    rgba.resize((size_t)w * h * 4);
    for (size_t i = 0; i < (size_t)w * h; ++i) {
        const uint8_t* p = &rgbe[4 * i];
        float* o = &rgba[4 * i];
        if (p[3] != 0) {
            const float f = (float)ldexp(1.0f, (int)p[3] - (int)(128 + 8));
            o[0] = p[0] * f;
            o[1] = p[1] * f;
            o[2] = p[2] * f;
        } else {
            o[0] = o[1] = o[2] = 0.0f;
        }
        o[3] = 1.0f;
    }
    return true;
}

uint32_t be32(const uint8_t* p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }

bool loadPNG(const std::string& data, std::vector<float>& rgba, uint32_t& w, uint32_t& h, std::string& err)
{
    static const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
    const uint8_t* d = (const uint8_t*)data.data();
    const size_t n = data.size();
    if (n < 8 || memcmp(d, sig, 8) != 0) { err = "not a PNG file"; return false; }
    size_t pos = 8;
    uint32_t depth = 0, ctype = 0, interlace = 0;
    std::vector<uint8_t> idat, plte, trns;
    bool haveHdr = false;
    while (pos + 8 <= n) {
        const uint32_t len = be32(d + pos);
        const std::string type((const char*)d + pos + 4, 4);
        if (pos + 12 + (size_t)len > n) { err = "truncated PNG chunk"; return false; }
        const uint8_t* c = d + pos + 8;
        if (type == "IHDR") {
            if (len < 13) { err = "bad IHDR"; return false; }
            w = be32(c);
            h = be32(c + 4);
            depth = c[8];
            ctype = c[9];
            interlace = c[12];
            haveHdr = true;
        } else if (type == "PLTE") {
            plte.assign(c, c + len);
        } else if (type == "tRNS") {
            trns.assign(c, c + len);
        } else if (type == "IDAT") {
            idat.insert(idat.end(), c, c + len);
        } else if (type == "IEND") {
            break;
        }
        pos += 12 + (size_t)len;
    }
    if (!haveHdr || w == 0 || h == 0 || w > (1u << 24) || h > (1u << 24)) { err = "bad PNG header"; return false; }
    if (interlace != 0) { err = "interlaced PNG not supported"; return false; }
    int channels;
    switch (ctype) {
    case 0: channels = 1; break;
    case 2: channels = 3; break;
    case 3: channels = 1; break;
    case 4: channels = 2; break;
    case 6: channels = 4; break;
    default: err = "bad PNG color type"; return false;
    }
    if (!(depth == 8 || depth == 16 || (ctype == 3 && (depth == 1 || depth == 2 || depth == 4)) ||
          (ctype == 0 && (depth == 1 || depth == 2 || depth == 4)))) {
        err = "unsupported PNG bit depth";
        return false;
    }
    const size_t bitsPerPixel = (size_t)channels * depth;
    const size_t stride = ((size_t)w * bitsPerPixel + 7) / 8;
    const size_t bpp = std::max<size_t>(1, bitsPerPixel / 8);
    std::vector<uint8_t> raw((stride + 1) * h);
    uLongf rawLen = (uLongf)raw.size();
    if (uncompress(raw.data(), &rawLen, idat.data(), (uLong)idat.size()) != Z_OK || rawLen != raw.size()) {
        err = "PNG inflate failed";
        return false;
    }
    std::vector<uint8_t> img(stride * h);
    for (uint32_t y = 0; y < h; ++y) {
        const uint8_t f = raw[y * (stride + 1)];
        const uint8_t* src = &raw[y * (stride + 1) + 1];
        uint8_t* cur = &img[y * stride];
        const uint8_t* prev = y ? &img[(y - 1) * stride] : nullptr;
        for (size_t i = 0; i < stride; ++i) {
            const int a = i >= bpp ? cur[i - bpp] : 0;
            const int b = prev ? prev[i] : 0;
            const int cc = (prev && i >= bpp) ? prev[i - bpp] : 0;
            int v = src[i];
            switch (f) {
            case 0: break;
            case 1: v += a; break;
            case 2: v += b; break;
            case 3: v += (a + b) >> 1; break;
            case 4: {
                const int p = a + b - cc, pa = abs(p - a), pb = abs(p - b), pc = abs(p - cc);
                v += (pa <= pb && pa <= pc) ? a : (pb <= pc ? b : cc);
                break;
            }
            default: err = "bad PNG filter"; return false;
            }
            cur[i] = (uint8_t)v;
        }
    }
    rgba.resize((size_t)w * h * 4);
    auto sample = [&](const uint8_t* row, uint32_t x, int ch) -> uint32_t {
        if (depth == 16) return row[(x * channels + ch) * 2];             // stb: 16 -> 8 bit keeps the high byte
        if (depth == 8) return row[x * channels + ch];
        const uint32_t bit = x * depth;
        const uint32_t v = (row[bit / 8] >> (8 - depth - bit % 8)) & ((1u << depth) - 1);
        if (ctype == 3) return v;
        return v * (255u / ((1u << depth) - 1));                           // gray expansion
    };
    for (uint32_t y = 0; y < h; ++y) {
        const uint8_t* row = &img[y * stride];
        for (uint32_t x = 0; x < w; ++x) {
            uint32_t r, g, b, a = 255;
            if (ctype == 3) {
                const uint32_t idx = sample(row, x, 0);
                if (3 * idx + 2 >= plte.size()) { err = "bad PNG palette index"; return false; }
                r = plte[3 * idx]; g = plte[3 * idx + 1]; b = plte[3 * idx + 2];
                if (idx < trns.size()) a = trns[idx];
            } else if (channels <= 2) {
                r = g = b = sample(row, x, 0);
                if (channels == 2) a = sample(row, x, 1);
            } else {
                r = sample(row, x, 0); g = sample(row, x, 1); b = sample(row, x, 2);
                if (channels == 4) a = sample(row, x, 3);
            }
            float* o = &rgba[4 * ((size_t)y * w + x)];
            o[0] = (float)r / 255.0f;
            o[1] = (float)g / 255.0f;
            o[2] = (float)b / 255.0f;
            o[3] = (float)a / 255.0f;
        }
    }
    return true;
}

void putBE32(std::string& s, uint32_t v)
{
    s += (char)(v >> 24);
    s += (char)(v >> 16);
    s += (char)(v >> 8);
    s += (char)v;
}

void chunk(std::string& out, const char* type, const std::string& data)
{
    putBE32(out, (uint32_t)data.size());
    std::string td = std::string(type, 4) + data;
    out += td;
    putBE32(out, (uint32_t)crc32(0, (const Bytef*)td.data(), (uInt)td.size()));
}

} // namespace

bool isHdrFile(const std::string& path)
{
    std::ifstream f(path, std::ios::binary);
    char head[11] = {0};
    f.read(head, 10);
    return strncmp(head, "#?RADIANCE", 10) == 0 || strncmp(head, "#?RGBE", 6) == 0;
}

bool loadImageRGBA32F(const std::string& path, std::vector<float>& rgba, uint32_t& w, uint32_t& h, std::string& err)
{
    std::string data;
    if (!readFile(path, data)) { err = "cannot open " + path; return false; }
    if (data.compare(0, 2, "#?") == 0) return loadHDR(data, rgba, w, h, err);
    return loadPNG(data, rgba, w, h, err);
}

bool writePNG(const std::string& path, uint32_t w, uint32_t h, const uint8_t* rgba, bool flip)
{
    std::string raw;
    raw.reserve((size_t)(4 * w + 1) * h);
    for (uint32_t y = 0; y < h; ++y) {
        const uint32_t sy = flip ? h - 1 - y : y;
        raw += (char)0;
        raw.append((const char*)rgba + (size_t)sy * w * 4, (size_t)w * 4);
    }
    uLongf clen = compressBound((uLong)raw.size());
    std::string comp(clen, '\0');
    if (compress2((Bytef*)&comp[0], &clen, (const Bytef*)raw.data(), (uLong)raw.size(), 6) != Z_OK) return false;
    comp.resize(clen);
    std::string out("\x89PNG\r\n\x1a\n", 8);
    std::string ihdr;
    putBE32(ihdr, w);
    putBE32(ihdr, h);
    ihdr += (char)8;   // bit depth
    ihdr += (char)6;   // RGBA
    ihdr += (char)0;
    ihdr += (char)0;
    ihdr += (char)0;
    chunk(out, "IHDR", ihdr);
    chunk(out, "IDAT", comp);
    chunk(out, "IEND", "");
    std::ofstream f(path, std::ios::binary | std::ios::trunc);
    if (!f.is_open()) return false;
    f.write(out.data(), (std::streamsize)out.size());
    return f.good();
}

bool writeHDR(const std::string& path, uint32_t w, uint32_t h, const float* rgba, bool flip)
{
    std::ofstream f(path, std::ios::binary | std::ios::trunc);
    if (!f.is_open()) return false;
    char head[160];
    snprintf(head, sizeof(head), "#?RADIANCE\n# Written by pathtracer_amd\nFORMAT=32-bit_rle_rgbe\nEXPOSURE=1.0\n\n-Y %u +X %u\n", h, w);
    f << head;
    std::vector<uint8_t> row((size_t)w * 4);
    for (uint32_t y = 0; y < h; ++y) {
        const uint32_t sy = flip ? h - 1 - y : y;
        for (uint32_t x = 0; x < w; ++x) {
            const float* l = rgba + 4 * ((size_t)sy * w + x);
            uint8_t* e = &row[4 * x];
            const float maxc = std::max(l[0], std::max(l[1], l[2]));     // stbiw__linear_to_rgbe
            if (maxc < 1e-32f) {
                e[0] = e[1] = e[2] = e[3] = 0;
            } else {
                int ex;
                const float nrm = (float)frexp(maxc, &ex) * 256.0f / maxc;
                e[0] = (uint8_t)(l[0] * nrm);
                e[1] = (uint8_t)(l[1] * nrm);
                e[2] = (uint8_t)(l[2] * nrm);
                e[3] = (uint8_t)(ex + 128);
            }
        }
        f.write((const char*)row.data(), (std::streamsize)row.size());
    }
    return f.good();
}

} // namespace ptamd
