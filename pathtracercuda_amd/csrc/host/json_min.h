// Minimal JSON reader for scene files: one flat, arena-allocated document (no per-value heap
// allocation, so a 30 MB scene parses and frees in a fraction of the time a node-per-value DOM
// takes).  Semantics follow what the reference's loader observes through nlohmann::json 3.9.0:
//  * a number token with '.', 'e' or 'E' is a float, others are integers (getFloat() accepts only
//    float tokens, SceneLoader.cpp:163-171); integer tokens are int64 or uint64 (nlohmann's
//    number_integer / number_unsigned), and one outside both becomes a float value;
//  * floats are converted correctly rounded to double (nlohmann's strtod) and narrowed by the caller;
//  * duplicate object keys: the last one wins (nlohmann's operator[] assignment);
//  * object key order is not observable by the loader (lookups only).
#pragma once
#include <cstdint>
#include <string>
#include <string_view>
#include <vector>

namespace ptamd {
namespace json {

enum class Kind : uint8_t { Null, Bool, Int, UInt, Float, String, Array, Object, Invalid };

struct Node {
    Kind kind = Kind::Null;
    bool b = false;
    uint32_t a = 0, n = 0;      // Array/Object: children kids[a, a+n); String: strings[a, a+n)
    double f = 0.0;
    int64_t i = 0;
    uint64_t u = 0;             // UInt: a non-negative integer token above INT64_MAX
};

struct Document {
    std::vector<Node> nodes;    // nodes[0] is the root
    std::vector<uint32_t> kids; // child node indices, contiguous per container
    std::vector<uint32_t> keyA, keyN;   // object keys of kids[k] (offset, length in strings)
    std::string strings;
};

// Read-only view of one value of a Document.
class Value {
public:
    Value() = default;
    Value(const Document* d, uint32_t idx) : d_(d), idx_(idx) {}
    bool valid() const { return d_ != nullptr; }
    Kind kind() const { return d_ ? d_->nodes[idx_].kind : Kind::Invalid; }
    bool isNumber() const { return kind() == Kind::Int || kind() == Kind::UInt || kind() == Kind::Float; }
    bool isFloat() const { return kind() == Kind::Float; }
    double f() const { return d_->nodes[idx_].f; }
    float asFloat() const
    {
        const Node& n = d_->nodes[idx_];
        if (n.kind == Kind::Float) return (float)n.f;
        if (n.kind == Kind::Int) return (float)n.i;
        return n.kind == Kind::UInt ? (float)n.u : 0.0f;
    }
    std::string_view str() const
    {
        const Node& n = d_->nodes[idx_];
        return std::string_view(d_->strings.data() + n.a, n.n);
    }
    uint32_t size() const { return (kind() == Kind::Array || kind() == Kind::Object) ? d_->nodes[idx_].n : 0u; }
    Value at(uint32_t k) const { return Value(d_, d_->kids[d_->nodes[idx_].a + k]); }
    // Object member (the last occurrence of `key`), or an invalid view.
    Value get(std::string_view key) const
    {
        if (kind() != Kind::Object) return Value();
        const Node& n = d_->nodes[idx_];
        for (uint32_t k = n.a + n.n; k-- > n.a;)
            if (std::string_view(d_->strings.data() + d_->keyA[k], d_->keyN[k]) == key) return Value(d_, d_->kids[k]);
        return Value();
    }

private:
    const Document* d_ = nullptr;
    uint32_t idx_ = 0;
};

// Returns false and sets `error` ("[json.exception.parse_error] ..."-style) on malformed input.
bool parse(std::string_view text, Document& out, std::string& error);
inline Value root(const Document& d) { return d.nodes.empty() ? Value() : Value(&d, 0); }

} // namespace json
} // namespace ptamd
