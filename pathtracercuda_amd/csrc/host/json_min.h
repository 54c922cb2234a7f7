// Minimal JSON DOM for scene files.  Numbers keep the distinction nlohmann::json 3.9.0 makes
// between integer and float tokens (a token with '.', 'e' or 'E' is a float): the reference's
// getFloat() accepts only float tokens (SceneLoader.cpp:163-171).  Floats are converted with
// strtod (correctly rounded, as nlohmann's lexer does) and narrowed to float by the caller.
#pragma once
#include <cstdint>
#include <map>
#include <memory>
#include <string>
#include <vector>

namespace ptamd {
namespace json {

struct Value {
    enum Kind { Null, Bool, Int, Float, String, Array, Object } kind = Null;
    bool b = false;
    int64_t i = 0;
    double f = 0.0;
    std::string s;
    std::vector<Value> arr;
    std::map<std::string, Value> obj;   // sorted, like nlohmann::json's default object_t

    bool isNumber() const { return kind == Int || kind == Float; }
    bool isFloat() const { return kind == Float; }
    float asFloat() const { return kind == Float ? (float)f : (kind == Int ? (float)i : 0.0f); }
    const Value* get(const char* key) const
    {
        if (kind != Object) return nullptr;
        auto it = obj.find(key);
        return it == obj.end() ? nullptr : &it->second;
    }
};

// Returns false and sets `error` ("[json.exception.parse_error] ..."-style) on malformed input.
bool parse(const std::string& text, Value& out, std::string& error);

} // namespace json
} // namespace ptamd
