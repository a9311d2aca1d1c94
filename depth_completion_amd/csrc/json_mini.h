// Minimal JSON reader for the native session's host side: safetensors headers, diffusers config.json files
// and the tuned GEMM table.  Values: null, bool, number (double), string, array, object (ordered keys).
// No external dependency; parse errors throw std::runtime_error with the byte offset.
#pragma once
#include <algorithm>
#include <cstdlib>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace dcjson {

struct Value {
  enum Kind { Null, Bool, Num, Str, Arr, Obj } kind = Null;
  bool b = false;
  double num = 0.0;
  std::string str;
  std::vector<Value> arr;
  std::vector<std::pair<std::string, Value>> obj;

  const Value* get(const std::string& k) const {
    if (kind != Obj) return nullptr;
    for (auto& kv : obj)
      if (kv.first == k) return &kv.second;
    return nullptr;
  }
  const Value& at(const std::string& k) const {
    const Value* v = get(k);
    if (!v) throw std::runtime_error("json: missing key '" + k + "'");
    return *v;
  }
  long long as_int() const {
    if (kind == Bool) return b ? 1 : 0;
    if (kind != Num) throw std::runtime_error("json: not a number");
    // |v| < 2^62: the conversion is defined, and sizes / offsets built from it cannot overflow a product
    if (!(num > -4.6e18 && num < 4.6e18)) throw std::runtime_error("json: integer out of range");
    return (long long)num;
  }
  double as_num() const {
    if (kind != Num) throw std::runtime_error("json: not a number");
    return num;
  }
};

class Parser {
 public:
  Parser(const char* s, size_t n) : s_(s), n_(n) {}
  Value parse() {
    Value v = value();
    ws();
    if (i_ != n_) fail("trailing characters");
    return v;
  }

 private:
  const char* s_;
  size_t n_, i_ = 0;
  int depth_ = 0;
  static constexpr int kMaxDepth = 128;  // nesting bound: a hostile header cannot exhaust the stack
  [[noreturn]] void fail(const char* what) {
    throw std::runtime_error(std::string("json: ") + what + " at byte " + std::to_string(i_));
  }
  void ws() {
    while (i_ < n_ && (s_[i_] == ' ' || s_[i_] == '\n' || s_[i_] == '\r' || s_[i_] == '\t')) ++i_;
  }
  bool lit(const char* w) {
    size_t k = 0;
    while (w[k]) {
      if (i_ + k >= n_ || s_[i_ + k] != w[k]) return false;
      ++k;
    }
    i_ += k;
    return true;
  }
  std::string string_() {
    if (i_ >= n_ || s_[i_] != '"') fail("expected string");
    ++i_;
    std::string out;
    while (i_ < n_ && s_[i_] != '"') {
      char c = s_[i_++];
      if (c == '\\') {
        if (i_ >= n_) fail("bad escape");
        char e = s_[i_++];
        switch (e) {
          case 'n': out += '\n'; break;
          case 't': out += '\t'; break;
          case 'r': out += '\r'; break;
          case 'b': out += '\b'; break;
          case 'f': out += '\f'; break;
          case 'u': {  // keep the code unit as UTF-8 (BMP only; enough for config files)
            if (i_ + 4 > n_) fail("bad \\u escape");
            unsigned cp = (unsigned)strtoul(std::string(s_ + i_, 4).c_str(), nullptr, 16);
            i_ += 4;
            if (cp < 0x80) {
              out += (char)cp;
            } else if (cp < 0x800) {
              out += (char)(0xC0 | (cp >> 6));
              out += (char)(0x80 | (cp & 0x3F));
            } else {
              out += (char)(0xE0 | (cp >> 12));
              out += (char)(0x80 | ((cp >> 6) & 0x3F));
              out += (char)(0x80 | (cp & 0x3F));
            }
            break;
          }
          default: out += e;
        }
      } else {
        out += c;
      }
    }
    if (i_ >= n_) fail("unterminated string");
    ++i_;
    return out;
  }
  Value value() {
    ws();
    if (i_ >= n_) fail("unexpected end");
    if (++depth_ > kMaxDepth) fail("nesting too deep");
    struct Leave {
      int& d;
      ~Leave() { --d; }
    } leave{depth_};
    Value v;
    char c = s_[i_];
    if (c == '{') {
      v.kind = Value::Obj;
      ++i_;
      ws();
      if (i_ < n_ && s_[i_] == '}') { ++i_; return v; }
      while (true) {
        ws();
        std::string k = string_();
        ws();
        if (i_ >= n_ || s_[i_] != ':') fail("expected ':'");
        ++i_;
        v.obj.emplace_back(std::move(k), value());
        ws();
        if (i_ < n_ && s_[i_] == ',') { ++i_; continue; }
        if (i_ < n_ && s_[i_] == '}') { ++i_; break; }
        fail("expected ',' or '}'");
      }
    } else if (c == '[') {
      v.kind = Value::Arr;
      ++i_;
      ws();
      if (i_ < n_ && s_[i_] == ']') { ++i_; return v; }
      while (true) {
        v.arr.push_back(value());
        ws();
        if (i_ < n_ && s_[i_] == ',') { ++i_; continue; }
        if (i_ < n_ && s_[i_] == ']') { ++i_; break; }
        fail("expected ',' or ']'");
      }
    } else if (c == '"') {
      v.kind = Value::Str;
      v.str = string_();
    } else if (lit("true")) {
      v.kind = Value::Bool;
      v.b = true;
    } else if (lit("false")) {
      v.kind = Value::Bool;
    } else if (lit("null")) {
      v.kind = Value::Null;
    } else {
      char* end = nullptr;
      std::string tmp(s_ + i_, std::min<size_t>(n_ - i_, 64));
      v.num = strtod(tmp.c_str(), &end);
      if (end == tmp.c_str()) fail("bad value");
      v.kind = Value::Num;
      i_ += (size_t)(end - tmp.c_str());
    }
    return v;
  }
};

inline Value parse(const std::string& s) { return Parser(s.data(), s.size()).parse(); }

}  // namespace dcjson
