// Native HTTP ingestion for smsgate-busd (``--http-listen``): the reference's
// ``POST /sms/raw`` contract (services/api_gateway/main.py:106-134, schemas.py:13-30)
// served from the broker's own event loop, so an accepted SMS is stored (and
// group-committed to the journal) without a second process or a client round trip.
//
// This header holds the request-independent parts, kept byte-compatible with the
// Python gateway (services/gateway.py, tests/test_http_ingest.py diffs the two):
//   * payload validation with pydantic's lax rules for RawSMSPayload
//     (device_id / message / sender: str; timestamp: int -- a JSON integer, an
//     integral float, a bool, or a numeric string with optional sign, surrounding
//     blanks, '_' digit separators and a zero fraction; source: str | null)
//     -> 422 with pydantic-style error items;
//   * the RawSMS mapping (msg_id = md5(message), body = message, date =
//     str(timestamp)) and its domain rules (sender / body non-empty, source in
//     {device, xml}) -> 400 {"detail": "Invalid payload"};
//   * RawSMS.model_dump_json() byte for byte (field order, pydantic's string
//     escaping: \" \\ \b \f \n \r \t, other controls as \u00xx, UTF-8 kept).
#pragma once

#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "json.hpp"
#include "mpack.hpp"

namespace ingest {

// ------------------------------------------------------------------- MD5 (RFC 1321)
class Md5 {
 public:
  static std::string hex(const std::string& data) {
    uint32_t h[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};
    const size_t n = data.size();
    const unsigned char* p = (const unsigned char*)data.data();
    size_t off = 0;
    for (; off + 64 <= n; off += 64) block(h, p + off);  // whole blocks in place
    unsigned char tail[128] = {0};                       // the rest + padding + bit length
    const size_t rem = n - off;
    memcpy(tail, p + off, rem);
    tail[rem] = 0x80;
    const size_t tl = rem + 1 + 8 <= 64 ? 64 : 128;
    const uint64_t bits = (uint64_t)n * 8u;
    for (int i = 0; i < 8; ++i) tail[tl - 8 + i] = (unsigned char)((bits >> (8 * i)) & 0xff);
    block(h, tail);
    if (tl == 128) block(h, tail + 64);
    static const char* hx = "0123456789abcdef";
    std::string out(32, '0');
    for (int i = 0; i < 4; ++i)
      for (int b = 0; b < 4; ++b) {
        const unsigned v = (h[i] >> (8 * b)) & 0xff;
        out[8 * i + 2 * b] = hx[v >> 4];
        out[8 * i + 2 * b + 1] = hx[v & 15];
      }
    return out;
  }

 private:
  static uint32_t rotl(uint32_t x, int c) { return (x << c) | (x >> (32 - c)); }
  static void block(uint32_t h[4], const unsigned char* p) {
    static const uint32_t K[64] = {
        0xd76aa478, 0xe8c7b756, 0x242070db, 0xc1bdceee, 0xf57c0faf, 0x4787c62a, 0xa8304613, 0xfd469501,
        0x698098d8, 0x8b44f7af, 0xffff5bb1, 0x895cd7be, 0x6b901122, 0xfd987193, 0xa679438e, 0x49b40821,
        0xf61e2562, 0xc040b340, 0x265e5a51, 0xe9b6c7aa, 0xd62f105d, 0x02441453, 0xd8a1e681, 0xe7d3fbc8,
        0x21e1cde6, 0xc33707d6, 0xf4d50d87, 0x455a14ed, 0xa9e3e905, 0xfcefa3f8, 0x676f02d9, 0x8d2a4c8a,
        0xfffa3942, 0x8771f681, 0x6d9d6122, 0xfde5380c, 0xa4beea44, 0x4bdecfa9, 0xf6bb4b60, 0xbebfbc70,
        0x289b7ec6, 0xeaa127fa, 0xd4ef3085, 0x04881d05, 0xd9d4d039, 0xe6db99e5, 0x1fa27cf8, 0xc4ac5665,
        0xf4292244, 0x432aff97, 0xab9423a7, 0xfc93a039, 0x655b59c3, 0x8f0ccc92, 0xffeff47d, 0x85845dd1,
        0x6fa87e4f, 0xfe2ce6e0, 0xa3014314, 0x4e0811a1, 0xf7537e82, 0xbd3af235, 0x2ad7d2bb, 0xeb86d391};
    static const int R[64] = {7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22,
                              5, 9,  14, 20, 5, 9,  14, 20, 5, 9,  14, 20, 5, 9,  14, 20,
                              4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23,
                              6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21};
    uint32_t w[16];
    for (int i = 0; i < 16; ++i)
      w[i] = (uint32_t)p[4 * i] | ((uint32_t)p[4 * i + 1] << 8) | ((uint32_t)p[4 * i + 2] << 16) |
             ((uint32_t)p[4 * i + 3] << 24);
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3];
    for (int i = 0; i < 64; ++i) {
      uint32_t f;
      int g;
      if (i < 16) { f = (b & c) | (~b & d); g = i; }
      else if (i < 32) { f = (d & b) | (~d & c); g = (5 * i + 1) % 16; }
      else if (i < 48) { f = b ^ c ^ d; g = (3 * i + 5) % 16; }
      else { f = c ^ (b | ~d); g = (7 * i) % 16; }
      const uint32_t t = d;
      d = c;
      c = b;
      b = b + rotl(a + f + K[i] + w[g], R[i]);
      a = t;
    }
    h[0] += a;
    h[1] += b;
    h[2] += c;
    h[3] += d;
  }
};

// ------------------------------------------------------- pydantic-compatible JSON strings
inline void py_str(std::string& o, const std::string& s) {
  o.push_back('"');
  for (unsigned char c : s) {
    switch (c) {
      case '"': o += "\\\""; break;
      case '\\': o += "\\\\"; break;
      case '\b': o += "\\b"; break;
      case '\f': o += "\\f"; break;
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

// ------------------------------------------------------------------ validation
struct FieldError {
  std::string type, field, msg;
};

// last occurrence of `key` in a JSON object (Python's json keeps the last duplicate)
inline const mp::Value* field(const mp::Value& obj, const char* key) {
  const mp::Value* found = nullptr;
  for (auto& kv : obj.m)
    if (kv.first.t == mp::Value::STR && kv.first.s == key) found = &kv.second;
  return found;
}

// pydantic lax int from a JSON string: blanks stripped, optional sign, digits with
// single '_' separators between digits, optional '.' followed by zeros only
inline bool int_from_string(const std::string& raw, int64_t& out) {
  size_t a = 0, b = raw.size();
  while (a < b && isspace((unsigned char)raw[a])) ++a;
  while (b > a && isspace((unsigned char)raw[b - 1])) --b;
  if (a == b) return false;
  bool neg = false;
  if (raw[a] == '+' || raw[a] == '-') neg = raw[a++] == '-';
  if (a == b || !isdigit((unsigned char)raw[a])) return false;
  __int128 v = 0;
  size_t i = a;
  for (; i < b && raw[i] != '.'; ++i) {
    const char c = raw[i];
    if (c == '_') {
      if (i + 1 >= b || !isdigit((unsigned char)raw[i + 1]) || !isdigit((unsigned char)raw[i - 1])) return false;
      continue;
    }
    if (!isdigit((unsigned char)c)) return false;
    v = v * 10 + (c - '0');
    if (v > (__int128)INT64_MAX + 1) return false;
  }
  if (i < b) {  // fraction: zeros only
    if (i + 1 == b) return false;
    for (++i; i < b; ++i)
      if (raw[i] != '0') return false;
  }
  if (neg) v = -v;
  if (v > INT64_MAX || v < INT64_MIN) return false;
  out = (int64_t)v;
  return true;
}

struct Payload {
  std::string device_id, message, sender;
  int64_t timestamp = 0;
  bool has_source = false;  // null / missing -> None
  std::string source;
};

// RawSMSPayload validation (FastAPI -> 422 on failure).  Returns false with errors.
inline bool validate_payload(const mp::Value& v, Payload& p, std::vector<FieldError>& errs) {
  if (v.t != mp::Value::MAP) {
    errs.push_back({"model_attributes_type", "", "Input should be a valid dictionary or object to extract fields from"});
    return false;
  }
  auto str_field = [&](const char* k, std::string& out) {
    const mp::Value* f = field(v, k);
    if (!f) errs.push_back({"missing", k, "Field required"});
    else if (f->t != mp::Value::STR) errs.push_back({"string_type", k, "Input should be a valid string"});
    else out = f->s;
  };
  str_field("device_id", p.device_id);
  str_field("message", p.message);
  str_field("sender", p.sender);
  const mp::Value* ts = field(v, "timestamp");
  if (!ts) {
    errs.push_back({"missing", "timestamp", "Field required"});
  } else if (ts->t == mp::Value::INT) {
    p.timestamp = ts->i;
  } else if (ts->t == mp::Value::BOOL) {
    p.timestamp = ts->b ? 1 : 0;
  } else if (ts->t == mp::Value::FLOAT) {
    if (std::isfinite(ts->f) && ts->f == std::floor(ts->f) && std::fabs(ts->f) < 9.2e18) p.timestamp = (int64_t)ts->f;
    else errs.push_back({"int_from_float", "timestamp", "Input should be a valid integer, got a number with a fractional part"});
  } else if (ts->t == mp::Value::STR) {
    if (!int_from_string(ts->s, p.timestamp))
      errs.push_back({"int_parsing", "timestamp", "Input should be a valid integer, unable to parse string as an integer"});
  } else {
    errs.push_back({"int_type", "timestamp", "Input should be a valid integer"});
  }
  const mp::Value* src = field(v, "source");
  if (src && src->t == mp::Value::STR) {
    p.has_source = true;
    p.source = src->s;
  } else if (src && src->t != mp::Value::NIL) {
    errs.push_back({"string_type", "source", "Input should be a valid string"});
  }
  return errs.empty();
}

// payload_to_raw + RawSMS.model_dump_json(); false = domain validation failed (400)
inline bool to_raw_json(const Payload& p, std::string& out) {
  if (p.sender.empty() || p.message.empty()) return false;
  if (!p.has_source || (p.source != "device" && p.source != "xml")) return false;
  out.clear();
  out += "{\"msg_id\":";
  py_str(out, Md5::hex(p.message));
  out += ",\"sender\":";
  py_str(out, p.sender);
  out += ",\"body\":";
  py_str(out, p.message);
  out += ",\"date\":";
  py_str(out, std::to_string(p.timestamp));
  out += ",\"device_id\":";
  py_str(out, p.device_id);
  out += ",\"source\":";
  py_str(out, p.source);
  out += "}";
  return true;
}

inline std::string errors_json(const std::vector<FieldError>& errs, long index = -1) {
  std::string o = "{\"detail\":[";
  for (size_t k = 0; k < errs.size(); ++k) {
    if (k) o.push_back(',');
    o += "{\"type\":";
    py_str(o, errs[k].type);
    o += ",\"loc\":[\"body\"";
    if (index >= 0) o += "," + std::to_string(index);
    if (!errs[k].field.empty()) {
      o.push_back(',');
      py_str(o, errs[k].field);
    }
    o += "],\"msg\":";
    py_str(o, errs[k].msg);
    o.push_back('}');
  }
  o += "]}";
  return o;
}

// One ingestion request: `batch` = POST /sms/raw/batch (a JSON array of payloads).
// status 202 with `raws` = the RawSMS JSON documents to store on sms.raw, or an
// error status (422 / 400) with its JSON body; nothing is stored unless every
// payload of a batch is valid (the Python gateway validates all before publishing).
struct Result {
  int status = 202;
  std::string body;
  std::vector<std::string> raws;
};

inline Result handle(const std::string& body, bool batch) {
  Result r;
  mp::Value v;
  try {
    v = json::parse(body);
  } catch (std::exception&) {
    r.status = 422;
    r.body = "{\"detail\":[{\"type\":\"json_invalid\",\"loc\":[\"body\"],\"msg\":\"JSON decode error\"}]}";
    return r;
  }
  std::vector<const mp::Value*> items;
  if (batch) {
    if (v.t != mp::Value::ARR) {
      r.status = 422;
      r.body = "{\"detail\":[{\"type\":\"list_type\",\"loc\":[\"body\"],\"msg\":\"Input should be a valid list\"}]}";
      return r;
    }
    for (auto& it : v.a) items.push_back(&it);
  } else {
    items.push_back(&v);
  }
  std::vector<Payload> ps(items.size());
  std::vector<FieldError> errs;
  std::string detail;
  for (size_t k = 0; k < items.size(); ++k) {
    std::vector<FieldError> e;
    if (!validate_payload(*items[k], ps[k], e)) {
      std::string one = errors_json(e, batch ? (long)k : -1);
      // merge the items' lists: strip {"detail":[ ... ]}
      one = one.substr(11, one.size() - 13);
      if (!detail.empty()) detail.push_back(',');
      detail += one;
    }
  }
  if (!detail.empty()) {
    r.status = 422;
    r.body = "{\"detail\":[" + detail + "]}";
    return r;
  }
  r.raws.resize(ps.size());
  for (size_t k = 0; k < ps.size(); ++k) {
    if (!to_raw_json(ps[k], r.raws[k])) {
      r.raws.clear();
      r.status = 400;
      r.body = "{\"detail\":\"Invalid payload\"}";
      return r;
    }
  }
  r.body = batch ? "{\"result\":\"queued\",\"count\":" + std::to_string(ps.size()) + "}" : "{\"result\":\"queued\"}";
  return r;
}

}  // namespace ingest
