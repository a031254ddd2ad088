// json.hpp -- flat-tape JSON reader for the objects crossing the C ABI.
// All values live in one std::vector<JVal>; containers link children by index, so a
// v1.Pod decodes with a handful of allocations.
#pragma once
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <string_view>
#include <vector>

namespace ksg {

struct JVal {
  enum Type : uint8_t { NUL, BOOL, NUM, STR, ARR, OBJ } type = NUL;
  bool b = false;
  std::string s;       // STR payload / NUM literal text / OBJ member key (in the child)
  std::string key;     // member name when this value sits inside an object
  int32_t first = -1;  // first child (ARR/OBJ)
  int32_t next = -1;   // next sibling
  int32_t count = 0;
};

class JDoc {
 public:
  JDoc(const char* p, size_t n) : p_(p), e_(p + n) {
    v_.reserve(64);
    root_ = parse_value();
    skip_ws();
    if (p_ != e_) throw std::runtime_error("json: trailing data");
  }
  const JVal& root() const { return v_[root_]; }
  const JVal& at(int32_t i) const { return v_[i]; }
  // member lookup; nullptr if absent or JSON null
  const JVal* get(const JVal& o, std::string_view k) const {
    if (o.type != JVal::OBJ) return nullptr;
    for (int32_t c = o.first; c >= 0; c = v_[c].next)
      if (v_[c].key == k) return v_[c].type == JVal::NUL ? nullptr : &v_[c];
    return nullptr;
  }
  bool present(const JVal& o, std::string_view k) const { return get(o, k) != nullptr; }
  std::string str(const JVal& o, std::string_view k, const char* def = "") const {
    const JVal* v = get(o, k);
    return (v && v->type == JVal::STR) ? v->s : std::string(def);
  }
  int64_t num(const JVal& o, std::string_view k, int64_t def = 0) const {
    const JVal* v = get(o, k);
    if (!v) return def;
    if (v->type == JVal::NUM || v->type == JVal::STR) return std::strtoll(v->s.c_str(), nullptr, 10);
    return def;
  }
  bool boolean(const JVal& o, std::string_view k) const {
    const JVal* v = get(o, k);
    return v && v->type == JVal::BOOL && v->b;
  }
  template <typename F>
  void each(const JVal* a, F f) const {  // array elements / object members
    if (!a || (a->type != JVal::ARR && a->type != JVal::OBJ)) return;
    for (int32_t c = a->first; c >= 0; c = v_[c].next) f(v_[c]);
  }

 private:
  const char* p_;
  const char* e_;
  std::vector<JVal> v_;
  int32_t root_ = -1;

  [[noreturn]] void fail(const char* m) { throw std::runtime_error(std::string("json: ") + m); }
  void skip_ws() {
    while (p_ < e_ && (*p_ == ' ' || *p_ == '\t' || *p_ == '\n' || *p_ == '\r')) ++p_;
  }
  static int hexv(char c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
  }
  uint32_t read_hex4() {
    if (e_ - p_ < 4) fail("short \\u");
    uint32_t v = 0;
    for (int i = 0; i < 4; ++i) {
      int h = hexv(*p_++);
      if (h < 0) fail("bad \\u");
      v = v * 16 + (uint32_t)h;
    }
    return v;
  }
  static void put_utf8(std::string& o, uint32_t cp) {
    if (cp < 0x80) {
      o.push_back((char)cp);
    } else if (cp < 0x800) {
      o.push_back((char)(0xC0 | (cp >> 6)));
      o.push_back((char)(0x80 | (cp & 0x3F)));
    } else if (cp < 0x10000) {
      o.push_back((char)(0xE0 | (cp >> 12)));
      o.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
      o.push_back((char)(0x80 | (cp & 0x3F)));
    } else {
      o.push_back((char)(0xF0 | (cp >> 18)));
      o.push_back((char)(0x80 | ((cp >> 12) & 0x3F)));
      o.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
      o.push_back((char)(0x80 | (cp & 0x3F)));
    }
  }
  std::string parse_string() {
    if (p_ >= e_ || *p_ != '"') fail("expected string");
    ++p_;
    const char* start = p_;
    while (p_ < e_ && *p_ != '"' && *p_ != '\\') ++p_;  // fast path: no escapes
    std::string out(start, p_);
    while (true) {
      if (p_ >= e_) fail("unterminated string");
      char c = *p_++;
      if (c == '"') return out;
      if (c != '\\') { out.push_back(c); continue; }
      if (p_ >= e_) fail("bad escape");
      char x = *p_++;
      switch (x) {
        case '"': out.push_back('"'); break;
        case '\\': out.push_back('\\'); break;
        case '/': out.push_back('/'); break;
        case 'b': out.push_back('\b'); break;
        case 'f': out.push_back('\f'); break;
        case 'n': out.push_back('\n'); break;
        case 'r': out.push_back('\r'); break;
        case 't': out.push_back('\t'); break;
        case 'u': {
          uint32_t cp = read_hex4();
          if (cp >= 0xD800 && cp <= 0xDBFF && e_ - p_ >= 6 && p_[0] == '\\' && p_[1] == 'u') {
            p_ += 2;
            uint32_t lo = read_hex4();
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          }
          put_utf8(out, cp);
          break;
        }
        default: fail("bad escape");
      }
    }
  }
  int32_t push(JVal&& v) {
    v_.push_back(std::move(v));
    return (int32_t)v_.size() - 1;
  }
  int32_t parse_value() {
    skip_ws();
    if (p_ >= e_) fail("unexpected end");
    const char c = *p_;
    if (c == '{' || c == '[') {
      const bool obj = c == '{';
      ++p_;
      JVal v;
      v.type = obj ? JVal::OBJ : JVal::ARR;
      int32_t self = push(std::move(v));
      int32_t prev = -1;
      skip_ws();
      if (p_ < e_ && *p_ == (obj ? '}' : ']')) { ++p_; return self; }
      while (true) {
        std::string key;
        if (obj) {
          skip_ws();
          key = parse_string();
          skip_ws();
          if (p_ >= e_ || *p_ != ':') fail("expected ':'");
          ++p_;
        }
        int32_t ch = parse_value();
        v_[ch].key = std::move(key);
        if (prev < 0) v_[self].first = ch;
        else v_[prev].next = ch;
        prev = ch;
        v_[self].count++;
        skip_ws();
        if (p_ < e_ && *p_ == ',') { ++p_; continue; }
        if (p_ < e_ && *p_ == (obj ? '}' : ']')) { ++p_; return self; }
        fail("expected ',' or closing bracket");
      }
    }
    JVal v;
    if (c == '"') {
      v.type = JVal::STR;
      v.s = parse_string();
    } else if (e_ - p_ >= 4 && std::memcmp(p_, "true", 4) == 0) {
      p_ += 4; v.type = JVal::BOOL; v.b = true;
    } else if (e_ - p_ >= 5 && std::memcmp(p_, "false", 5) == 0) {
      p_ += 5; v.type = JVal::BOOL;
    } else if (e_ - p_ >= 4 && std::memcmp(p_, "null", 4) == 0) {
      p_ += 4; v.type = JVal::NUL;
    } else {
      const char* q = p_;
      while (q < e_ && (std::strchr("+-0123456789.eE", *q) != nullptr) && *q) ++q;
      if (q == p_) fail("unexpected character");
      v.type = JVal::NUM;
      v.s.assign(p_, q);
      p_ = q;
    }
    return push(std::move(v));
  }
};

}  // namespace ksg
