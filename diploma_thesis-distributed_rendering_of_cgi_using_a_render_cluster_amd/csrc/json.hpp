// Minimal JSON reader for .rrscene files (objects, arrays, numbers, strings,
// true/false/null). Numbers are parsed with strtod (exact round trip of the
// exporter's repr() output). Not a general-purpose library: no \u surrogate
// pairs beyond the BMP, no streaming.
#pragma once

#include <cmath>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace rr {

struct Json {
    enum Type { Null, Bool, Number, String, Array, Object } type = Null;
    bool b = false;
    double num = 0.0;
    std::string str;
    std::vector<Json> arr;
    std::map<std::string, Json> obj;

    bool has(const std::string& k) const { return type == Object && obj.count(k) != 0; }
    const Json& operator[](const std::string& k) const {
        auto it = obj.find(k);
        if (type != Object || it == obj.end()) throw std::runtime_error("missing key '" + k + "'");
        return it->second;
    }
    const Json& operator[](size_t i) const {
        if (type != Array || i >= arr.size()) throw std::runtime_error("array index out of range");
        return arr[i];
    }
    size_t size() const { return type == Array ? arr.size() : (type == Object ? obj.size() : 0); }
    double as_num() const {
        if (type == Bool) return b ? 1.0 : 0.0;
        if (type != Number) throw std::runtime_error("expected number");
        return num;
    }
    const std::string& as_str() const {
        if (type != String) throw std::runtime_error("expected string");
        return str;
    }
    double get_num(const std::string& k, double dflt) const {
        return has(k) && (*this)[k].type != Null ? (*this)[k].as_num() : dflt;
    }
    std::string get_str(const std::string& k, const std::string& dflt) const {
        return has(k) && (*this)[k].type == String ? (*this)[k].str : dflt;
    }
};

class JsonParser {
public:
    explicit JsonParser(const std::string& text) : s_(text.c_str()), p_(text.c_str()) {}
    Json parse() {
        Json v = value();
        ws();
        if (*p_) fail("trailing characters");
        return v;
    }

private:
    const char* s_;
    const char* p_;

    [[noreturn]] void fail(const char* what) {
        throw std::runtime_error(std::string("JSON parse error at offset ") +
                                 std::to_string(p_ - s_) + ": " + what);
    }
    void ws() {
        while (*p_ == ' ' || *p_ == '\n' || *p_ == '\r' || *p_ == '\t') ++p_;
    }
    Json value() {
        ws();
        Json v;
        switch (*p_) {
            case '{': {
                v.type = Json::Object;
                ++p_;
                ws();
                if (*p_ == '}') { ++p_; return v; }
                for (;;) {
                    ws();
                    if (*p_ != '"') fail("expected key");
                    std::string k = string();
                    ws();
                    if (*p_ != ':') fail("expected ':'");
                    ++p_;
                    v.obj[k] = value();
                    ws();
                    if (*p_ == ',') { ++p_; continue; }
                    if (*p_ == '}') { ++p_; return v; }
                    fail("expected ',' or '}'");
                }
            }
            case '[': {
                v.type = Json::Array;
                ++p_;
                ws();
                if (*p_ == ']') { ++p_; return v; }
                for (;;) {
                    v.arr.push_back(value());
                    ws();
                    if (*p_ == ',') { ++p_; continue; }
                    if (*p_ == ']') { ++p_; return v; }
                    fail("expected ',' or ']'");
                }
            }
            case '"':
                v.type = Json::String;
                v.str = string();
                return v;
            case 't':
                if (strncmp(p_, "true", 4) != 0) fail("bad literal");
                p_ += 4; v.type = Json::Bool; v.b = true; return v;
            case 'f':
                if (strncmp(p_, "false", 5) != 0) fail("bad literal");
                p_ += 5; v.type = Json::Bool; v.b = false; return v;
            case 'n':
                if (strncmp(p_, "null", 4) != 0) fail("bad literal");
                p_ += 4; return v;
            case 'N':  // Python json writes NaN/Infinity; accept them
                if (strncmp(p_, "NaN", 3) != 0) fail("bad literal");
                p_ += 3; v.type = Json::Number; v.num = std::nan(""); return v;
            case 'I':
                if (strncmp(p_, "Infinity", 8) != 0) fail("bad literal");
                p_ += 8; v.type = Json::Number; v.num = HUGE_VAL; return v;
            default: {
                char* end = nullptr;
                if (strncmp(p_, "-Infinity", 9) == 0) {
                    p_ += 9; v.type = Json::Number; v.num = -HUGE_VAL; return v;
                }
                double d = strtod(p_, &end);
                if (end == p_) fail("unexpected character");
                p_ = end;
                v.type = Json::Number;
                v.num = d;
                return v;
            }
        }
    }
    std::string string() {
        std::string out;
        ++p_;  // opening quote
        while (*p_ && *p_ != '"') {
            if (*p_ == '\\') {
                ++p_;
                switch (*p_) {
                    case 'n': out += '\n'; break;
                    case 't': out += '\t'; break;
                    case 'r': out += '\r'; break;
                    case 'b': out += '\b'; break;
                    case 'f': out += '\f'; break;
                    case 'u': {
                        unsigned cp = (unsigned)strtoul(std::string(p_ + 1, 4).c_str(), nullptr, 16);
                        p_ += 4;
                        if (cp < 0x80) out += (char)cp;
                        else if (cp < 0x800) { out += (char)(0xC0 | (cp >> 6)); out += (char)(0x80 | (cp & 0x3F)); }
                        else { out += (char)(0xE0 | (cp >> 12)); out += (char)(0x80 | ((cp >> 6) & 0x3F)); out += (char)(0x80 | (cp & 0x3F)); }
                        break;
                    }
                    default: out += *p_; break;
                }
                ++p_;
            } else {
                out += *p_++;
            }
        }
        if (*p_ != '"') fail("unterminated string");
        ++p_;
        return out;
    }
};

}  // namespace rr
