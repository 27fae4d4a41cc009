// Minimal MessagePack value model + codec for the native broker.
//
// Covers exactly what the bus wire protocol and the journal use (the Python
// side is ``msgpack.packb(..., use_bin_type=True)`` / ``unpackb(raw=False)``):
// nil, bool, signed/unsigned ints, float32/64, str, bin, array, map.
#pragma once

#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace mp {

struct Value {
  enum Type : uint8_t { NIL, BOOL, INT, FLOAT, STR, BIN, ARR, MAP };
  Type t = NIL;
  bool b = false;
  int64_t i = 0;
  double f = 0.0;
  std::string s;                                // STR / BIN payload
  std::vector<Value> a;                         // ARR
  std::vector<std::pair<Value, Value>> m;       // MAP

  Value() = default;
  static Value nil() { return Value(); }
  static Value boolean(bool v) { Value x; x.t = BOOL; x.b = v; return x; }
  static Value integer(int64_t v) { Value x; x.t = INT; x.i = v; return x; }
  static Value real(double v) { Value x; x.t = FLOAT; x.f = v; return x; }
  static Value str(std::string v) { Value x; x.t = STR; x.s = std::move(v); return x; }
  static Value bin(std::string v) { Value x; x.t = BIN; x.s = std::move(v); return x; }
  static Value arr() { Value x; x.t = ARR; return x; }
  static Value map() { Value x; x.t = MAP; return x; }

  bool is_nil() const { return t == NIL; }
  int64_t as_int() const {
    if (t == INT) return i;
    if (t == FLOAT) return (int64_t)f;
    if (t == BOOL) return b ? 1 : 0;
    throw std::runtime_error("expected an integer");
  }
  double as_double() const {
    if (t == FLOAT) return f;
    if (t == INT) return (double)i;
    throw std::runtime_error("expected a number");
  }
  const std::string& as_str() const {
    if (t != STR && t != BIN) throw std::runtime_error("expected a string");
    return s;
  }
  const std::vector<Value>& as_arr() const {
    if (t != ARR) throw std::runtime_error("expected an array");
    return a;
  }
  const Value* get(const char* key) const {  // map lookup by string key
    if (t != MAP) return nullptr;
    for (auto& kv : m)
      if (kv.first.t == STR && kv.first.s == key) return &kv.second;
    return nullptr;
  }
  Value& push(Value v) { a.push_back(std::move(v)); return a.back(); }
  void put(const char* k, Value v) { m.emplace_back(Value::str(k), std::move(v)); }
};

// ------------------------------------------------------------------ encoding
inline void put_be(std::string& o, uint64_t v, int n) {
  for (int k = n - 1; k >= 0; --k) o.push_back((char)((v >> (8 * k)) & 0xff));
}

inline void enc_int(std::string& o, int64_t v) {
  if (v >= 0) {
    if (v < 128) o.push_back((char)v);
    else if (v < 256) { o.push_back((char)0xcc); put_be(o, v, 1); }
    else if (v < 65536) { o.push_back((char)0xcd); put_be(o, v, 2); }
    else if (v <= 0xffffffffLL) { o.push_back((char)0xce); put_be(o, v, 4); }
    else { o.push_back((char)0xcf); put_be(o, (uint64_t)v, 8); }
  } else {
    if (v >= -32) o.push_back((char)(int8_t)v);
    else if (v >= -128) { o.push_back((char)0xd0); put_be(o, (uint8_t)(int8_t)v, 1); }
    else if (v >= -32768) { o.push_back((char)0xd1); put_be(o, (uint16_t)(int16_t)v, 2); }
    else if (v >= INT32_MIN) { o.push_back((char)0xd2); put_be(o, (uint32_t)(int32_t)v, 4); }
    else { o.push_back((char)0xd3); put_be(o, (uint64_t)v, 8); }
  }
}

inline void enc_double(std::string& o, double d) {
  uint64_t u;
  std::memcpy(&u, &d, 8);
  o.push_back((char)0xcb);
  put_be(o, u, 8);
}

inline void enc_str(std::string& o, const char* p, size_t n) {
  if (n < 32) o.push_back((char)(0xa0 | n));
  else if (n < 256) { o.push_back((char)0xd9); put_be(o, n, 1); }
  else if (n < 65536) { o.push_back((char)0xda); put_be(o, n, 2); }
  else { o.push_back((char)0xdb); put_be(o, n, 4); }
  o.append(p, n);
}
inline void enc_str(std::string& o, const std::string& s) { enc_str(o, s.data(), s.size()); }

inline void enc_bin(std::string& o, const char* p, size_t n) {
  if (n < 256) { o.push_back((char)0xc4); put_be(o, n, 1); }
  else if (n < 65536) { o.push_back((char)0xc5); put_be(o, n, 2); }
  else { o.push_back((char)0xc6); put_be(o, n, 4); }
  o.append(p, n);
}

inline void enc_arr_hdr(std::string& o, size_t n) {
  if (n < 16) o.push_back((char)(0x90 | n));
  else if (n < 65536) { o.push_back((char)0xdc); put_be(o, n, 2); }
  else { o.push_back((char)0xdd); put_be(o, n, 4); }
}

inline void enc_map_hdr(std::string& o, size_t n) {
  if (n < 16) o.push_back((char)(0x80 | n));
  else if (n < 65536) { o.push_back((char)0xde); put_be(o, n, 2); }
  else { o.push_back((char)0xdf); put_be(o, n, 4); }
}

inline void enc_nil(std::string& o) { o.push_back((char)0xc0); }
inline void enc_bool(std::string& o, bool b) { o.push_back(b ? (char)0xc3 : (char)0xc2); }

inline void encode(std::string& o, const Value& v) {
  switch (v.t) {
    case Value::NIL: enc_nil(o); break;
    case Value::BOOL: enc_bool(o, v.b); break;
    case Value::INT: enc_int(o, v.i); break;
    case Value::FLOAT: enc_double(o, v.f); break;
    case Value::STR: enc_str(o, v.s); break;
    case Value::BIN: enc_bin(o, v.s.data(), v.s.size()); break;
    case Value::ARR:
      enc_arr_hdr(o, v.a.size());
      for (auto& x : v.a) encode(o, x);
      break;
    case Value::MAP:
      enc_map_hdr(o, v.m.size());
      for (auto& kv : v.m) { encode(o, kv.first); encode(o, kv.second); }
      break;
  }
}

// ------------------------------------------------------------------ decoding
struct Reader {
  const uint8_t* p;
  const uint8_t* end;
  int depth = 0;

  uint64_t be(int n) {
    need(n);
    uint64_t v = 0;
    for (int k = 0; k < n; ++k) v = (v << 8) | p[k];
    p += n;
    return v;
  }
  void need(size_t n) const {
    if ((size_t)(end - p) < n) throw std::runtime_error("truncated msgpack");
  }
  std::string bytes(size_t n) {
    need(n);
    std::string s((const char*)p, n);
    p += n;
    return s;
  }
  Value read() {
    if (++depth > 64) throw std::runtime_error("msgpack nesting too deep");
    Value v = read_inner();
    --depth;
    return v;
  }
  Value read_arr(size_t n) {
    Value v = Value::arr();
    v.a.reserve(n < 4096 ? n : 4096);
    for (size_t k = 0; k < n; ++k) v.a.push_back(read());
    return v;
  }
  Value read_map(size_t n) {
    Value v = Value::map();
    for (size_t k = 0; k < n; ++k) {
      Value key = read();
      Value val = read();
      v.m.emplace_back(std::move(key), std::move(val));
    }
    return v;
  }
  Value read_inner() {
    need(1);
    uint8_t c = *p++;
    if (c <= 0x7f) return Value::integer(c);
    if (c >= 0xe0) return Value::integer((int8_t)c);
    if ((c & 0xe0) == 0xa0) return Value::str(bytes(c & 0x1f));
    if ((c & 0xf0) == 0x90) return read_arr(c & 0x0f);
    if ((c & 0xf0) == 0x80) return read_map(c & 0x0f);
    switch (c) {
      case 0xc0: return Value::nil();
      case 0xc2: return Value::boolean(false);
      case 0xc3: return Value::boolean(true);
      case 0xc4: { size_t n = be(1); return Value::bin(bytes(n)); }
      case 0xc5: { size_t n = be(2); return Value::bin(bytes(n)); }
      case 0xc6: { size_t n = be(4); return Value::bin(bytes(n)); }
      case 0xca: { uint32_t u = (uint32_t)be(4); float f; std::memcpy(&f, &u, 4); return Value::real(f); }
      case 0xcb: { uint64_t u = be(8); double d; std::memcpy(&d, &u, 8); return Value::real(d); }
      case 0xcc: return Value::integer((int64_t)be(1));
      case 0xcd: return Value::integer((int64_t)be(2));
      case 0xce: return Value::integer((int64_t)be(4));
      case 0xcf: return Value::integer((int64_t)be(8));
      case 0xd0: return Value::integer((int8_t)be(1));
      case 0xd1: return Value::integer((int16_t)be(2));
      case 0xd2: return Value::integer((int32_t)be(4));
      case 0xd3: return Value::integer((int64_t)be(8));
      case 0xd9: { size_t n = be(1); return Value::str(bytes(n)); }
      case 0xda: { size_t n = be(2); return Value::str(bytes(n)); }
      case 0xdb: { size_t n = be(4); return Value::str(bytes(n)); }
      case 0xdc: return read_arr(be(2));
      case 0xdd: return read_arr(be(4));
      case 0xde: return read_map(be(2));
      case 0xdf: return read_map(be(4));
      default: throw std::runtime_error("unsupported msgpack type byte");
    }
  }
};

inline Value decode(const void* data, size_t n) {
  Reader r{(const uint8_t*)data, (const uint8_t*)data + n};
  Value v = r.read();
  if (r.p != r.end) throw std::runtime_error("trailing bytes after msgpack value");
  return v;
}

}  // namespace mp

// ---------------------------------------------------------------------- CRC-32
// zlib-compatible CRC-32 (reflected 0xEDB88320), slicing-by-8: the journal
// frames are ``[u32 len][u32 zlib.crc32(body)][body]`` on both sides.
namespace crc {

struct Tables {
  uint32_t t[8][256];
  Tables() {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c & 1) ? (0xEDB88320u ^ (c >> 1)) : (c >> 1);
      t[0][i] = c;
    }
    for (uint32_t i = 0; i < 256; ++i)
      for (int s = 1; s < 8; ++s) t[s][i] = (t[s - 1][i] >> 8) ^ t[0][t[s - 1][i] & 0xff];
  }
};

inline const Tables& tables() {
  static const Tables T;
  return T;
}

inline uint32_t crc32(const void* data, size_t n, uint32_t crc = 0) {
  const Tables& T = tables();
  const uint8_t* p = (const uint8_t*)data;
  crc = ~crc;
  while (n >= 8) {
    uint32_t lo, hi;
    std::memcpy(&lo, p, 4);
    std::memcpy(&hi, p + 4, 4);
    lo ^= crc;
    crc = T.t[7][lo & 0xff] ^ T.t[6][(lo >> 8) & 0xff] ^ T.t[5][(lo >> 16) & 0xff] ^ T.t[4][lo >> 24] ^
          T.t[3][hi & 0xff] ^ T.t[2][(hi >> 8) & 0xff] ^ T.t[1][(hi >> 16) & 0xff] ^ T.t[0][hi >> 24];
    p += 8;
    n -= 8;
  }
  while (n--) crc = T.t[0][(crc ^ *p++) & 0xff] ^ (crc >> 8);
  return ~crc;
}

}  // namespace crc
