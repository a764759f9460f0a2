// otr_json.h — minimal JSON DOM reader/writer for the drop-in JSON entry points
// (trace request body Batch.java:56-65 / reporter_service.py:184-205, and the
// Match()/report() response bodies README.md:269-302).
#pragma once
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "otr_request.h"

namespace otrjson {

struct Value;
using Ptr = std::shared_ptr<Value>;

struct Value {
  enum Kind { Null, Bool, Number, String, Array, Object } kind = Null;
  bool b = false;
  double num = 0;
  bool is_int = false;
  int64_t i = 0;
  std::string str;
  std::vector<Ptr> arr;
  std::vector<std::pair<std::string, Ptr>> obj;

  const Value* get(const char* k) const {
    if (kind != Object) return nullptr;
    for (auto& kv : obj)
      if (kv.first == k) return kv.second.get();
    return nullptr;
  }
  double as_double() const { return is_int ? (double)i : num; }
  int64_t as_int() const { return is_int ? i : (int64_t)num; }
};

class Parser {
 public:
  Parser(const char* s, size_t n) : p_(s), e_(s + n) {}
  Ptr parse(std::string* err) {
    Ptr v = value();
    ws();
    if (!v || (p_ != e_ && *p_ != '\0')) {
      if (err) *err = err_.empty() ? "invalid JSON" : err_;
      return nullptr;
    }
    return v;
  }

 private:
  const char* p_;
  const char* e_;
  std::string err_;
  int depth_ = 0;
  void ws() {
    while (p_ < e_ && (*p_ == ' ' || *p_ == '\t' || *p_ == '\n' || *p_ == '\r')) ++p_;
  }
  Ptr fail(const char* m) {
    if (err_.empty()) err_ = m;
    return nullptr;
  }
  Ptr value() {
    ws();
    if (p_ >= e_) return fail("unexpected end of JSON");
    if (++depth_ > 256) return fail("JSON nested too deeply");
    Ptr r;
    char c = *p_;
    if (c == '{') r = object();
    else if (c == '[') r = array();
    else if (c == '"') {
      r = std::make_shared<Value>();
      r->kind = Value::String;
      if (!string(&r->str)) r = nullptr;
    } else if (c == 't' && e_ - p_ >= 4 && !strncmp(p_, "true", 4)) {
      p_ += 4;
      r = std::make_shared<Value>();
      r->kind = Value::Bool;
      r->b = true;
    } else if (c == 'f' && e_ - p_ >= 5 && !strncmp(p_, "false", 5)) {
      p_ += 5;
      r = std::make_shared<Value>();
      r->kind = Value::Bool;
    } else if (c == 'n' && e_ - p_ >= 4 && !strncmp(p_, "null", 4)) {
      p_ += 4;
      r = std::make_shared<Value>();
    } else r = number();
    --depth_;
    return r;
  }
  Ptr number() {
    const char* s = p_;
    if (p_ < e_ && (*p_ == '-' || *p_ == '+')) ++p_;
    bool frac = false;
    while (p_ < e_ && ((*p_ >= '0' && *p_ <= '9') || *p_ == '.' || *p_ == 'e' || *p_ == 'E' ||
                       ((*p_ == '-' || *p_ == '+') && (p_[-1] == 'e' || p_[-1] == 'E')))) {
      if (*p_ == '.' || *p_ == 'e' || *p_ == 'E') frac = true;
      ++p_;
    }
    if (p_ == s) return fail("invalid JSON value");
    std::string tok(s, p_ - s);
    auto v = std::make_shared<Value>();
    v->kind = Value::Number;
    char* end = nullptr;
    if (!frac) {
      errno = 0;
      long long x = strtoll(tok.c_str(), &end, 10);
      if (errno == 0 && end && *end == '\0') {
        v->is_int = true;
        v->i = x;
        v->num = (double)x;
        return v;
      }
    }
    v->num = strtod(tok.c_str(), &end);  // correctly rounded (glibc)
    if (!end || *end != '\0') return fail("invalid JSON number");
    return v;
  }
  bool string(std::string* out) {
    ++p_;
    while (p_ < e_ && *p_ != '"') {
      char c = *p_++;
      if (c == '\\') {
        if (p_ >= e_) return false;
        char x = *p_++;
        switch (x) {
          case '"': out->push_back('"'); break;
          case '\\': out->push_back('\\'); break;
          case '/': out->push_back('/'); break;
          case 'b': out->push_back('\b'); break;
          case 'f': out->push_back('\f'); break;
          case 'n': out->push_back('\n'); break;
          case 'r': out->push_back('\r'); break;
          case 't': out->push_back('\t'); break;
          case 'u': {
            if (e_ - p_ < 4) return false;
            unsigned cp = (unsigned)strtoul(std::string(p_, 4).c_str(), nullptr, 16);
            p_ += 4;
            if (cp < 0x80) out->push_back((char)cp);
            else if (cp < 0x800) {
              out->push_back((char)(0xC0 | (cp >> 6)));
              out->push_back((char)(0x80 | (cp & 0x3F)));
            } else {
              out->push_back((char)(0xE0 | (cp >> 12)));
              out->push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
              out->push_back((char)(0x80 | (cp & 0x3F)));
            }
            break;
          }
          default: return false;
        }
      } else {
        out->push_back(c);
      }
    }
    if (p_ >= e_) return false;
    ++p_;
    return true;
  }
  Ptr array() {
    ++p_;
    auto v = std::make_shared<Value>();
    v->kind = Value::Array;
    ws();
    if (p_ < e_ && *p_ == ']') {
      ++p_;
      return v;
    }
    for (;;) {
      Ptr x = value();
      if (!x) return nullptr;
      v->arr.push_back(x);
      ws();
      if (p_ < e_ && *p_ == ',') { ++p_; continue; }
      if (p_ < e_ && *p_ == ']') { ++p_; return v; }
      return fail("invalid JSON array");
    }
  }
  Ptr object() {
    ++p_;
    auto v = std::make_shared<Value>();
    v->kind = Value::Object;
    ws();
    if (p_ < e_ && *p_ == '}') {
      ++p_;
      return v;
    }
    for (;;) {
      ws();
      if (p_ >= e_ || *p_ != '"') return fail("invalid JSON object key");
      std::string k;
      if (!string(&k)) return fail("invalid JSON string");
      ws();
      if (p_ >= e_ || *p_ != ':') return fail("invalid JSON object");
      ++p_;
      Ptr x = value();
      if (!x) return nullptr;
      v->obj.emplace_back(std::move(k), x);
      ws();
      if (p_ < e_ && *p_ == ',') { ++p_; continue; }
      if (p_ < e_ && *p_ == '}') { ++p_; return v; }
      return fail("invalid JSON object");
    }
  }
};

// shortest round-tripping repr of a double, Python-style ("1000.0", "1e-05")
// repr() digits and layout, as json.dumps prints floats (reporter_service.py:243)
inline void put_double(std::string& o, double v) { otrreq::put_repr(o, v); }

inline void put_string(std::string& o, const std::string& s) {
  o.push_back('"');
  for (unsigned char c : s) {
    switch (c) {
      case '"': o += "\\\""; break;
      case '\\': o += "\\\\"; break;
      case '\n': o += "\\n"; break;
      case '\r': o += "\\r"; break;
      case '\t': o += "\\t"; break;
      default:
        if (c < 0x20) {
          char b[8];
          snprintf(b, sizeof b, "\\u%04x", c);
          o += b;
        } else {
          o.push_back((char)c);
        }
    }
  }
  o.push_back('"');
}

inline void put_value(std::string& o, const Value& v) {
  switch (v.kind) {
    case Value::Null: o += "null"; break;
    case Value::Bool: o += v.b ? "true" : "false"; break;
    case Value::Number:
      if (v.is_int) o += std::to_string(v.i);
      else put_double(o, v.num);
      break;
    case Value::String: put_string(o, v.str); break;
    case Value::Array:
      o.push_back('[');
      for (size_t k = 0; k < v.arr.size(); ++k) {
        if (k) o.push_back(',');
        put_value(o, *v.arr[k]);
      }
      o.push_back(']');
      break;
    case Value::Object:
      o.push_back('{');
      for (size_t k = 0; k < v.obj.size(); ++k) {
        if (k) o.push_back(',');
        put_string(o, v.obj[k].first);
        o.push_back(':');
        put_value(o, *v.obj[k].second);
      }
      o.push_back('}');
      break;
  }
}

}  // namespace otrjson
