// minijson.hpp -- tiny JSON DOM used by the parity oracle (test infrastructure only).
// Generic RFC 8259 reader: objects keep key order, numbers keep their source text so
// integer fields are read exactly (no double round trip).
#pragma once
#include <cstdint>
#include <cstdlib>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace mj {

struct Value {
  enum Kind { Null, Bool, Number, String, Array, Object } kind = Null;
  bool b = false;
  std::string s;  // String payload, or the literal text of a Number
  std::vector<Value> arr;
  std::vector<std::pair<std::string, Value>> obj;

  bool is_null() const { return kind == Null; }
  bool is_obj() const { return kind == Object; }
  bool is_arr() const { return kind == Array; }
  bool is_str() const { return kind == String; }
  const Value* get(const std::string& k) const {
    if (kind != Object) return nullptr;
    for (auto& kv : obj)
      if (kv.first == k) return &kv.second;
    return nullptr;
  }
  // present and not JSON null
  const Value* has(const std::string& k) const {
    const Value* v = get(k);
    return (v && v->kind != Null) ? v : nullptr;
  }
  std::string str(const std::string& k, const std::string& def = "") const {
    const Value* v = get(k);
    return (v && v->kind == String) ? v->s : def;
  }
  int64_t i64(const std::string& k, int64_t def = 0) const {
    const Value* v = get(k);
    if (!v) return def;
    if (v->kind == Number) return std::strtoll(v->s.c_str(), nullptr, 10);
    if (v->kind == String) return std::strtoll(v->s.c_str(), nullptr, 10);
    return def;
  }
  bool boolean(const std::string& k, bool def = false) const {
    const Value* v = get(k);
    return (v && v->kind == Bool) ? v->b : def;
  }
};

class Parser {
 public:
  Parser(const char* p, size_t n) : p_(p), e_(p + n) {}
  Value parse() {
    Value v = value();
    ws();
    if (p_ != e_) fail("trailing characters");
    return v;
  }

 private:
  const char* p_;
  const char* e_;
  [[noreturn]] void fail(const char* m) { throw std::runtime_error(std::string("json: ") + m); }
  void ws() {
    while (p_ < e_ && (*p_ == ' ' || *p_ == '\n' || *p_ == '\r' || *p_ == '\t')) ++p_;
  }
  bool lit(const char* s) {
    const char* q = p_;
    while (*s) {
      if (q >= e_ || *q != *s) return false;
      ++q, ++s;
    }
    p_ = q;
    return true;
  }
  static void utf8(std::string& out, uint32_t cp) {
    if (cp < 0x80) out += char(cp);
    else if (cp < 0x800) { out += char(0xC0 | (cp >> 6)); out += char(0x80 | (cp & 0x3F)); }
    else if (cp < 0x10000) {
      out += char(0xE0 | (cp >> 12)); out += char(0x80 | ((cp >> 6) & 0x3F)); out += char(0x80 | (cp & 0x3F));
    } else {
      out += char(0xF0 | (cp >> 18)); out += char(0x80 | ((cp >> 12) & 0x3F));
      out += char(0x80 | ((cp >> 6) & 0x3F)); out += char(0x80 | (cp & 0x3F));
    }
  }
  uint32_t hex4() {
    if (e_ - p_ < 4) fail("bad \\u escape");
    uint32_t v = 0;
    for (int i = 0; i < 4; ++i) {
      char c = *p_++;
      v <<= 4;
      if (c >= '0' && c <= '9') v |= c - '0';
      else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
      else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
      else fail("bad hex digit");
    }
    return v;
  }
  std::string string() {
    if (p_ >= e_ || *p_ != '"') fail("expected string");
    ++p_;
    std::string out;
    while (true) {
      if (p_ >= e_) fail("unterminated string");
      char c = *p_++;
      if (c == '"') break;
      if (c != '\\') { out += c; continue; }
      if (p_ >= e_) fail("bad escape");
      char x = *p_++;
      switch (x) {
        case '"': out += '"'; break;
        case '\\': out += '\\'; break;
        case '/': out += '/'; break;
        case 'b': out += '\b'; break;
        case 'f': out += '\f'; break;
        case 'n': out += '\n'; break;
        case 'r': out += '\r'; break;
        case 't': out += '\t'; break;
        case 'u': {
          uint32_t cp = hex4();
          if (cp >= 0xD800 && cp < 0xDC00 && e_ - p_ >= 6 && p_[0] == '\\' && p_[1] == 'u') {
            p_ += 2;
            uint32_t lo = hex4();
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          }
          utf8(out, cp);
          break;
        }
        default: fail("bad escape");
      }
    }
    return out;
  }
  Value value() {
    ws();
    if (p_ >= e_) fail("unexpected end");
    Value v;
    char c = *p_;
    if (c == '{') {
      ++p_;
      v.kind = Value::Object;
      ws();
      if (p_ < e_ && *p_ == '}') { ++p_; return v; }
      while (true) {
        ws();
        std::string k = string();
        ws();
        if (p_ >= e_ || *p_ != ':') fail("expected ':'");
        ++p_;
        v.obj.emplace_back(std::move(k), value());
        ws();
        if (p_ < e_ && *p_ == ',') { ++p_; continue; }
        if (p_ < e_ && *p_ == '}') { ++p_; break; }
        fail("expected ',' or '}'");
      }
    } else if (c == '[') {
      ++p_;
      v.kind = Value::Array;
      ws();
      if (p_ < e_ && *p_ == ']') { ++p_; return v; }
      while (true) {
        v.arr.push_back(value());
        ws();
        if (p_ < e_ && *p_ == ',') { ++p_; continue; }
        if (p_ < e_ && *p_ == ']') { ++p_; break; }
        fail("expected ',' or ']'");
      }
    } else if (c == '"') {
      v.kind = Value::String;
      v.s = string();
    } else if (lit("true")) {
      v.kind = Value::Bool; v.b = true;
    } else if (lit("false")) {
      v.kind = Value::Bool; v.b = false;
    } else if (lit("null")) {
      v.kind = Value::Null;
    } else {
      const char* q = p_;
      if (q < e_ && (*q == '-' || *q == '+')) ++q;
      while (q < e_ && ((*q >= '0' && *q <= '9') || *q == '.' || *q == 'e' || *q == 'E' || *q == '-' || *q == '+')) ++q;
      if (q == p_) fail("unexpected character");
      v.kind = Value::Number;
      v.s.assign(p_, q);
      p_ = q;
    }
    return v;
  }
};

inline Value parse(const char* p, size_t n) { return Parser(p, n).parse(); }

}  // namespace mj
