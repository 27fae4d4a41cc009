// Minimal JSON <-> mp::Value for the broker's NATS front-end (JetStream API bodies).
//
// Objects become MAP values with STR keys (insertion order kept), arrays ARR,
// integers INT (int64: JetStream durations are nanoseconds), other numbers FLOAT.
// Parsing throws std::runtime_error on malformed input; dumping writes compact JSON
// (BIN values are written as strings).
#pragma once

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <string>

#include "mpack.hpp"

namespace json {

class Parser {
 public:
  Parser(const char* p, size_t n) : p_(p), end_(p + n) {}

  mp::Value parse() {
    mp::Value v = value(0);
    ws();
    if (p_ != end_) fail("trailing characters");
    return v;
  }

 private:
  [[noreturn]] void fail(const char* what) { throw std::runtime_error(std::string("bad JSON: ") + what); }

  void ws() {
    while (p_ < end_ && (*p_ == ' ' || *p_ == '\t' || *p_ == '\n' || *p_ == '\r')) ++p_;
  }

  bool lit(const char* s) {
    size_t n = strlen(s);
    if ((size_t)(end_ - p_) >= n && memcmp(p_, s, n) == 0) {
      p_ += n;
      return true;
    }
    return false;
  }

  mp::Value value(int depth) {
    if (depth > 64) fail("nesting too deep");
    ws();
    if (p_ >= end_) fail("unexpected end");
    char c = *p_;
    if (c == '{') return object(depth);
    if (c == '[') return array(depth);
    if (c == '"') return mp::Value::str(string());
    if (lit("true")) return mp::Value::boolean(true);
    if (lit("false")) return mp::Value::boolean(false);
    if (lit("null")) return mp::Value::nil();
    return number();
  }

  mp::Value object(int depth) {
    ++p_;
    mp::Value v = mp::Value::map();
    ws();
    if (p_ < end_ && *p_ == '}') {
      ++p_;
      return v;
    }
    for (;;) {
      ws();
      if (p_ >= end_ || *p_ != '"') fail("expected a key");
      std::string k = string();
      ws();
      if (p_ >= end_ || *p_ != ':') fail("expected ':'");
      ++p_;
      v.m.emplace_back(mp::Value::str(std::move(k)), value(depth + 1));
      ws();
      if (p_ < end_ && *p_ == ',') {
        ++p_;
        continue;
      }
      if (p_ < end_ && *p_ == '}') {
        ++p_;
        return v;
      }
      fail("expected ',' or '}'");
    }
  }

  mp::Value array(int depth) {
    ++p_;
    mp::Value v = mp::Value::arr();
    ws();
    if (p_ < end_ && *p_ == ']') {
      ++p_;
      return v;
    }
    for (;;) {
      v.push(value(depth + 1));
      ws();
      if (p_ < end_ && *p_ == ',') {
        ++p_;
        continue;
      }
      if (p_ < end_ && *p_ == ']') {
        ++p_;
        return v;
      }
      fail("expected ',' or ']'");
    }
  }

  static void utf8(std::string& o, uint32_t cp) {
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

  uint32_t hex4() {
    if (end_ - p_ < 4) fail("short \\u escape");
    uint32_t v = 0;
    for (int k = 0; k < 4; ++k) {
      char c = *p_++;
      v <<= 4;
      if (c >= '0' && c <= '9') v |= (uint32_t)(c - '0');
      else if (c >= 'a' && c <= 'f') v |= (uint32_t)(c - 'a' + 10);
      else if (c >= 'A' && c <= 'F') v |= (uint32_t)(c - 'A' + 10);
      else fail("bad \\u escape");
    }
    return v;
  }

  std::string string() {
    ++p_;  // opening quote
    std::string o;
    while (p_ < end_ && *p_ != '"') {
      char c = *p_++;
      if (c != '\\') {
        o.push_back(c);
        continue;
      }
      if (p_ >= end_) fail("bad escape");
      char e = *p_++;
      switch (e) {
        case '"': o.push_back('"'); break;
        case '\\': o.push_back('\\'); break;
        case '/': o.push_back('/'); break;
        case 'b': o.push_back('\b'); break;
        case 'f': o.push_back('\f'); break;
        case 'n': o.push_back('\n'); break;
        case 'r': o.push_back('\r'); break;
        case 't': o.push_back('\t'); break;
        case 'u': {
          uint32_t cp = hex4();
          if (cp >= 0xD800 && cp < 0xDC00 && end_ - p_ >= 6 && p_[0] == '\\' && p_[1] == 'u') {
            p_ += 2;
            uint32_t lo = hex4();
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          }
          utf8(o, cp);
          break;
        }
        default: fail("bad escape");
      }
    }
    if (p_ >= end_) fail("unterminated string");
    ++p_;
    return o;
  }

  mp::Value number() {
    const char* s = p_;
    bool real = false;
    if (p_ < end_ && (*p_ == '-' || *p_ == '+')) ++p_;
    while (p_ < end_ && ((*p_ >= '0' && *p_ <= '9') || *p_ == '.' || *p_ == 'e' || *p_ == 'E' || *p_ == '-' ||
                         *p_ == '+')) {
      if (*p_ == '.' || *p_ == 'e' || *p_ == 'E') real = true;
      ++p_;
    }
    if (p_ == s) fail("unexpected character");
    std::string t(s, p_);
    char* e = nullptr;
    if (!real) {
      long long v = strtoll(t.c_str(), &e, 10);
      if (*e == 0) return mp::Value::integer(v);
    }
    double d = strtod(t.c_str(), &e);
    if (*e != 0) fail("bad number");
    return mp::Value::real(d);
  }

  const char* p_;
  const char* end_;
};

inline mp::Value parse(const std::string& s) { return Parser(s.data(), s.size()).parse(); }

inline void dump_str(std::string& o, const std::string& s) {
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

inline void dump(std::string& o, const mp::Value& v) {
  switch (v.t) {
    case mp::Value::NIL: o += "null"; break;
    case mp::Value::BOOL: o += v.b ? "true" : "false"; break;
    case mp::Value::INT: o += std::to_string(v.i); break;
    case mp::Value::FLOAT: {
      if (!std::isfinite(v.f)) {
        o += "null";
        break;
      }
      char b[32];
      snprintf(b, sizeof b, "%.17g", v.f);
      o += b;
      break;
    }
    case mp::Value::STR:
    case mp::Value::BIN: dump_str(o, v.s); break;
    case mp::Value::ARR: {
      o.push_back('[');
      for (size_t k = 0; k < v.a.size(); ++k) {
        if (k) o.push_back(',');
        dump(o, v.a[k]);
      }
      o.push_back(']');
      break;
    }
    case mp::Value::MAP: {
      o.push_back('{');
      for (size_t k = 0; k < v.m.size(); ++k) {
        if (k) o.push_back(',');
        dump_str(o, v.m[k].first.t == mp::Value::STR ? v.m[k].first.s : std::string("?"));
        o.push_back(':');
        dump(o, v.m[k].second);
      }
      o.push_back('}');
      break;
    }
  }
}

inline std::string dumps(const mp::Value& v) {
  std::string o;
  dump(o, v);
  return o;
}

}  // namespace json
