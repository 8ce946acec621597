// Minimal JSON reader for config.json and safetensors headers.
// Host-only; no exceptions escape the C ABI (capi.cpp converts them to status codes).
#pragma once
#include <cstdint>
#include <cstdlib>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace dsocr {

struct Json {
    enum Kind { Null, Bool, Number, String, Array, Object } kind = Null;
    bool b = false;
    double num = 0.0;
    std::string str;
    std::vector<Json> arr;
    std::map<std::string, Json> obj;

    bool is_null() const { return kind == Null; }
    bool has(const std::string& k) const { return kind == Object && obj.count(k) && !obj.at(k).is_null(); }
    const Json& operator[](const std::string& k) const {
        static const Json null_json;
        if (kind != Object) return null_json;
        auto it = obj.find(k);
        return it == obj.end() ? null_json : it->second;
    }
    const Json& operator[](size_t i) const { return arr.at(i); }
    size_t size() const { return kind == Array ? arr.size() : (kind == Object ? obj.size() : 0); }
    int64_t as_int(int64_t def = 0) const { return kind == Number ? (int64_t)num : (kind == Bool ? (int64_t)b : def); }
    double as_double(double def = 0.0) const { return kind == Number ? num : def; }
    bool as_bool(bool def = false) const { return kind == Bool ? b : (kind == Number ? num != 0.0 : def); }
    std::string as_string(const std::string& def = "") const { return kind == String ? str : def; }

    static Json parse(const char* p, size_t n) {
        const char* end = p + n;
        Json j = parse_value(p, end);
        skip_ws(p, end);
        return j;
    }
    static Json parse(const std::string& s) { return parse(s.data(), s.size()); }

  private:
    static void skip_ws(const char*& p, const char* e) {
        while (p < e && (*p == ' ' || *p == '\n' || *p == '\r' || *p == '\t')) ++p;
    }
    static void expect(const char*& p, const char* e, char c) {
        skip_ws(p, e);
        if (p >= e || *p != c) throw std::runtime_error(std::string("json: expected '") + c + "'");
        ++p;
    }
    static std::string parse_string(const char*& p, const char* e) {
        expect(p, e, '"');
        std::string out;
        while (p < e && *p != '"') {
            if (*p == '\\') {
                ++p;
                if (p >= e) break;
                char c = *p++;
                switch (c) {
                    case 'n': out += '\n'; break;
                    case 't': out += '\t'; break;
                    case 'r': out += '\r'; break;
                    case 'b': out += '\b'; break;
                    case 'f': out += '\f'; break;
                    case 'u': {
                        if (e - p < 4) throw std::runtime_error("json: bad \\u escape");
                        unsigned cp = (unsigned)strtoul(std::string(p, 4).c_str(), nullptr, 16);
                        p += 4;
                        if (cp < 0x80) out += (char)cp;
                        else if (cp < 0x800) { out += (char)(0xC0 | (cp >> 6)); out += (char)(0x80 | (cp & 0x3F)); }
                        else { out += (char)(0xE0 | (cp >> 12)); out += (char)(0x80 | ((cp >> 6) & 0x3F)); out += (char)(0x80 | (cp & 0x3F)); }
                        break;
                    }
                    default: out += c;
                }
            } else {
                out += *p++;
            }
        }
        if (p >= e) throw std::runtime_error("json: unterminated string");
        ++p;
        return out;
    }
    static Json parse_value(const char*& p, const char* e) {
        skip_ws(p, e);
        if (p >= e) throw std::runtime_error("json: unexpected end");
        Json j;
        char c = *p;
        if (c == '{') {
            ++p;
            j.kind = Object;
            skip_ws(p, e);
            if (p < e && *p == '}') { ++p; return j; }
            while (true) {
                std::string k = parse_string(p, e);
                expect(p, e, ':');
                j.obj[k] = parse_value(p, e);
                skip_ws(p, e);
                if (p < e && *p == ',') { ++p; continue; }
                expect(p, e, '}');
                break;
            }
        } else if (c == '[') {
            ++p;
            j.kind = Array;
            skip_ws(p, e);
            if (p < e && *p == ']') { ++p; return j; }
            while (true) {
                j.arr.push_back(parse_value(p, e));
                skip_ws(p, e);
                if (p < e && *p == ',') { ++p; continue; }
                expect(p, e, ']');
                break;
            }
        } else if (c == '"') {
            j.kind = String;
            j.str = parse_string(p, e);
        } else if (c == 't' && e - p >= 4 && std::string(p, 4) == "true") {
            j.kind = Bool; j.b = true; p += 4;
        } else if (c == 'f' && e - p >= 5 && std::string(p, 5) == "false") {
            j.kind = Bool; j.b = false; p += 5;
        } else if (c == 'n' && e - p >= 4 && std::string(p, 4) == "null") {
            p += 4;
        } else {
            char* q = nullptr;
            std::string tmp(p, std::min<size_t>(64, (size_t)(e - p)));
            double v = strtod(tmp.c_str(), &q);
            if (q == tmp.c_str()) throw std::runtime_error("json: bad token");
            j.kind = Number; j.num = v;
            p += (q - tmp.c_str());
        }
        return j;
    }
};

}  // namespace dsocr
