// Recursive-descent JSON parser (RFC 8259) building a flat Document (json_min.h).
#include "json_min.h"

#include <charconv>
#include <cstdio>
#include <cstdlib>

namespace ptamd {
namespace json {
namespace {

struct Child {
    uint32_t node, keyA, keyN;
};

struct Parser {
    const char* p;
    const char* begin;
    const char* end;
    Document& d;
    std::vector<Child> scratch;     // children of the containers being parsed (a stack of ranges)
    std::string err;
    int depth = 0;

    bool fail(const char* what)
    {
        if (err.empty()) {
            char buf[256];
            snprintf(buf, sizeof(buf), "[json.exception.parse_error] parse error at byte %ld: %s",
                     (long)(p - begin) + 1, what);
            err = buf;
        }
        return false;
    }
    void ws()
    {
        while (p < end && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) ++p;
    }
    bool lit(const char* s)
    {
        const char* q = p;
        while (*s) {
            if (q >= end || *q != *s) return false;
            ++q;
            ++s;
        }
        p = q;
        return true;
    }
    void utf8(uint32_t cp)
    {
        std::string& o = d.strings;
        if (cp < 0x80) o += (char)cp;
        else if (cp < 0x800) { o += (char)(0xC0 | (cp >> 6)); o += (char)(0x80 | (cp & 0x3F)); }
        else if (cp < 0x10000) {
            o += (char)(0xE0 | (cp >> 12)); o += (char)(0x80 | ((cp >> 6) & 0x3F)); o += (char)(0x80 | (cp & 0x3F));
        } else {
            o += (char)(0xF0 | (cp >> 18)); o += (char)(0x80 | ((cp >> 12) & 0x3F));
            o += (char)(0x80 | ((cp >> 6) & 0x3F)); o += (char)(0x80 | (cp & 0x3F));
        }
    }
    bool hex4(uint32_t& v)
    {
        v = 0;
        for (int k = 0; k < 4; ++k) {
            if (p >= end) return fail("truncated \\u escape");
            char c = *p++;
            v <<= 4;
            if (c >= '0' && c <= '9') v |= (uint32_t)(c - '0');
            else if (c >= 'a' && c <= 'f') v |= (uint32_t)(c - 'a' + 10);
            else if (c >= 'A' && c <= 'F') v |= (uint32_t)(c - 'A' + 10);
            else return fail("invalid \\u escape");
        }
        return true;
    }
    // Appends the unescaped string to the arena; returns its (offset, length).
    bool str(uint32_t& a, uint32_t& n)
    {
        if (p >= end || *p != '"') return fail("expected string");
        ++p;
        a = (uint32_t)d.strings.size();
        while (true) {
            const char* run = p;                           // copy escape-free runs in one go
            while (p < end && *p != '"' && *p != '\\' && (unsigned char)*p >= 0x20) ++p;
            d.strings.append(run, (size_t)(p - run));
            if (p >= end) return fail("unterminated string");
            const unsigned char c = (unsigned char)*p++;
            if (c == '"') break;
            if (c < 0x20) return fail("control character in string");
            if (p >= end) return fail("unterminated escape");
            const char e = *p++;
            switch (e) {
            case '"': d.strings += '"'; break;
            case '\\': d.strings += '\\'; break;
            case '/': d.strings += '/'; break;
            case 'b': d.strings += '\b'; break;
            case 'f': d.strings += '\f'; break;
            case 'n': d.strings += '\n'; break;
            case 'r': d.strings += '\r'; break;
            case 't': d.strings += '\t'; break;
            case 'u': {
                uint32_t cp;
                if (!hex4(cp)) return false;
                if (cp >= 0xD800 && cp <= 0xDBFF) {
                    uint32_t lo;
                    if (!(lit("\\u") && hex4(lo)) || lo < 0xDC00 || lo > 0xDFFF) return fail("invalid surrogate pair");
                    cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
                } else if (cp >= 0xDC00 && cp <= 0xDFFF) {
                    return fail("invalid surrogate");
                }
                utf8(cp);
                break;
            }
            default: return fail("invalid escape");
            }
        }
        n = (uint32_t)(d.strings.size() - a);
        return true;
    }
    bool num(Node& v)
    {
        const char* s = p;
        bool isFloat = false;
        if (p < end && *p == '-') ++p;
        if (p >= end) return fail("invalid number");
        if (*p == '0') ++p;
        else if (*p >= '1' && *p <= '9') { while (p < end && *p >= '0' && *p <= '9') ++p; }
        else return fail("invalid number");
        if (p < end && *p == '.') {
            isFloat = true;
            ++p;
            if (p >= end || !(*p >= '0' && *p <= '9')) return fail("invalid number");
            while (p < end && *p >= '0' && *p <= '9') ++p;
        }
        if (p < end && (*p == 'e' || *p == 'E')) {
            isFloat = true;
            ++p;
            if (p < end && (*p == '+' || *p == '-')) ++p;
            if (p >= end || !(*p >= '0' && *p <= '9')) return fail("invalid number");
            while (p < end && *p >= '0' && *p <= '9') ++p;
        }
        if (!isFloat) {
            int64_t iv = 0;
            const auto r = std::from_chars(s, p, iv);
            if (r.ec == std::errc() && r.ptr == p) {
                v.kind = Kind::Int;
                v.i = iv;
                return true;
            }
            uint64_t uv = 0;
            const auto ru = std::from_chars(s, p, uv);
            if (ru.ec == std::errc() && ru.ptr == p) {
                v.kind = Kind::UInt;
                v.u = uv;
                return true;
            }
            // beyond uint64: nlohmann stores it as a float value (still an integer token)
        }
        double fv = 0.0;
        const auto r = std::from_chars(s, p, fv);          // correctly rounded, like strtod
        if (r.ec == std::errc::result_out_of_range) fv = strtod(std::string(s, p).c_str(), nullptr);   // +-inf / 0
        v.kind = Kind::Float;
        v.f = fv;
        return true;
    }
    bool value(uint32_t idx)
    {
        if (++depth > 512) return fail("nesting too deep");
        ws();
        if (p >= end) return fail("unexpected end of input");
        bool ok = true;
        switch (*p) {
        case '{':
        case '[': {
            const bool isObj = *p == '{';
            const char close = isObj ? '}' : ']';
            ++p;
            d.nodes[idx].kind = isObj ? Kind::Object : Kind::Array;
            const size_t first = scratch.size();
            ws();
            if (p < end && *p == close) { ++p; break; }
            while (true) {
                Child c{0, 0, 0};
                if (isObj) {
                    ws();
                    if (!str(c.keyA, c.keyN)) { ok = false; break; }
                    ws();
                    if (p >= end || *p != ':') { ok = fail("expected ':'"); break; }
                    ++p;
                }
                c.node = (uint32_t)d.nodes.size();
                d.nodes.emplace_back();
                if (!value(c.node)) { ok = false; break; }
                scratch.push_back(c);
                ws();
                if (p < end && *p == ',') { ++p; continue; }
                if (p < end && *p == close) { ++p; break; }
                ok = fail(isObj ? "expected ',' or '}'" : "expected ',' or ']'");
                break;
            }
            if (ok) {
                Node& n = d.nodes[idx];
                n.a = (uint32_t)d.kids.size();
                n.n = (uint32_t)(scratch.size() - first);
                for (size_t k = first; k < scratch.size(); ++k) {
                    d.kids.push_back(scratch[k].node);
                    d.keyA.push_back(scratch[k].keyA);
                    d.keyN.push_back(scratch[k].keyN);
                }
            }
            scratch.resize(first);
            break;
        }
        case '"': {
            uint32_t a = 0, n = 0;
            ok = str(a, n);
            Node& v = d.nodes[idx];
            v.kind = Kind::String;
            v.a = a;
            v.n = n;
            break;
        }
        case 't':
            if (lit("true")) { d.nodes[idx].kind = Kind::Bool; d.nodes[idx].b = true; }
            else ok = fail("invalid literal");
            break;
        case 'f':
            if (lit("false")) { d.nodes[idx].kind = Kind::Bool; d.nodes[idx].b = false; }
            else ok = fail("invalid literal");
            break;
        case 'n':
            if (lit("null")) d.nodes[idx].kind = Kind::Null;
            else ok = fail("invalid literal");
            break;
        default: {
            Node v;
            ok = num(v);
            d.nodes[idx] = v;
        }
        }
        --depth;
        return ok;
    }
};

} // namespace

bool parse(std::string_view text, Document& out, std::string& error)
{
    out = Document();
    out.nodes.reserve(text.size() / 8 + 16);
    out.kids.reserve(text.size() / 8 + 16);
    out.keyA.reserve(text.size() / 8 + 16);
    out.keyN.reserve(text.size() / 8 + 16);
    Parser ps{text.data(), text.data(), text.data() + text.size(), out, {}, {}};
    // skip a UTF-8 BOM like nlohmann does
    if (text.size() >= 3 && (unsigned char)text[0] == 0xEF && (unsigned char)text[1] == 0xBB && (unsigned char)text[2] == 0xBF)
        ps.p += 3;
    out.nodes.emplace_back();
    if (!ps.value(0)) { error = ps.err; return false; }
    ps.ws();
    if (ps.p != ps.end) { ps.fail("unexpected trailing characters"); error = ps.err; return false; }
    return true;
}

} // namespace json
} // namespace ptamd
