// Recursive-descent JSON parser (RFC 8259) for the scene loader.
#include "json_min.h"

#include <cerrno>
#include <cstdio>
#include <cstdlib>

namespace ptamd {
namespace json {
namespace {

struct Parser {
    const char* p;
    const char* begin;
    const char* end;
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
    static void utf8(std::string& o, uint32_t cp)
    {
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
    bool str(std::string& o)
    {
        if (p >= end || *p != '"') return fail("expected string");
        ++p;
        while (true) {
            if (p >= end) return fail("unterminated string");
            unsigned char c = (unsigned char)*p++;
            if (c == '"') return true;
            if (c < 0x20) return fail("control character in string");
            if (c != '\\') { o += (char)c; continue; }
            if (p >= end) return fail("unterminated escape");
            char e = *p++;
            switch (e) {
            case '"': o += '"'; break;
            case '\\': o += '\\'; break;
            case '/': o += '/'; break;
            case 'b': o += '\b'; break;
            case 'f': o += '\f'; break;
            case 'n': o += '\n'; break;
            case 'r': o += '\r'; break;
            case 't': o += '\t'; break;
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
                utf8(o, cp);
                break;
            }
            default: return fail("invalid escape");
            }
        }
    }
    bool num(Value& v)
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
        std::string tok(s, p);
        if (!isFloat) {
            errno = 0;
            char* e = nullptr;
            long long iv = strtoll(tok.c_str(), &e, 10);
            if (errno == 0 && e && *e == 0) {
                v.kind = Value::Int;
                v.i = iv;
                return true;
            }
            // out of int64 range: nlohmann stores it as a float value (still an integer token)
        }
        v.kind = Value::Float;
        v.f = strtod(tok.c_str(), nullptr);
        return true;
    }
    bool value(Value& v)
    {
        if (++depth > 512) return fail("nesting too deep");
        ws();
        if (p >= end) return fail("unexpected end of input");
        bool ok;
        switch (*p) {
        case '{': {
            ++p;
            v.kind = Value::Object;
            ws();
            if (p < end && *p == '}') { ++p; ok = true; break; }
            ok = true;
            while (true) {
                ws();
                std::string key;
                if (!str(key)) { ok = false; break; }
                ws();
                if (p >= end || *p != ':') { ok = fail("expected ':'"); break; }
                ++p;
                Value child;
                if (!value(child)) { ok = false; break; }
                v.obj[key] = std::move(child);
                ws();
                if (p < end && *p == ',') { ++p; continue; }
                if (p < end && *p == '}') { ++p; break; }
                ok = fail("expected ',' or '}'");
                break;
            }
            break;
        }
        case '[': {
            ++p;
            v.kind = Value::Array;
            ws();
            if (p < end && *p == ']') { ++p; ok = true; break; }
            ok = true;
            while (true) {
                Value child;
                if (!value(child)) { ok = false; break; }
                v.arr.push_back(std::move(child));
                ws();
                if (p < end && *p == ',') { ++p; continue; }
                if (p < end && *p == ']') { ++p; break; }
                ok = fail("expected ',' or ']'");
                break;
            }
            break;
        }
        case '"':
            v.kind = Value::String;
            ok = str(v.s);
            break;
        case 't':
            ok = lit("true") ? (v.kind = Value::Bool, v.b = true, true) : fail("invalid literal");
            break;
        case 'f':
            ok = lit("false") ? (v.kind = Value::Bool, v.b = false, true) : fail("invalid literal");
            break;
        case 'n':
            ok = lit("null") ? (v.kind = Value::Null, true) : fail("invalid literal");
            break;
        default:
            ok = num(v);
        }
        --depth;
        return ok;
    }
};

} // namespace

bool parse(const std::string& text, Value& out, std::string& error)
{
    Parser ps{text.data(), text.data(), text.data() + text.size(), {}};
    // skip a UTF-8 BOM like nlohmann does
    if (text.size() >= 3 && (unsigned char)text[0] == 0xEF && (unsigned char)text[1] == 0xBB && (unsigned char)text[2] == 0xBF)
        ps.p += 3;
    out = Value();
    if (!ps.value(out)) { error = ps.err; return false; }
    ps.ws();
    if (ps.p != ps.end) { ps.fail("unexpected trailing characters"); error = ps.err; return false; }
    return true;
}

} // namespace json
} // namespace ptamd
