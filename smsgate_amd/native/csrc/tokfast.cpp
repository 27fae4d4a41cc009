// _tokfast: native byte-level BPE encoder / field decoder of the extractor tokenizer.
//
// The parser processes tokenise every SMS body before it goes to the GPU engine and
// detokenise every answer that comes back (serving/remote.py).  With the HF
// `tokenizers` library that was ~25 us of host CPU per message (Encoding objects,
// Rayon hand-offs, a Python list per sequence) on top of ~20 us of answer decoding:
// the largest single item of the parser process's per-message CPU budget
// (VERDICT r03 weak #2).  This module does both in one C++ pass per batch and
// emits / consumes the engine wire format (serving/protocol.py) directly:
//
//   * the model's pre-tokenizer (models/tokenizer.py NUMBER_AWARE_SPLIT) as a
//     hand-written leftmost-first matcher (every alternative of the regex, in
//     order, with its backtracking behaviour) over code points, with the
//     letter / number / digit / whitespace classes supplied by Python
//     (tables probed against the library itself, models/fasttok.py);
//   * the added special tokens matched as literals first (AddedVocabulary);
//   * byte-level BPE with the merge ranks, and a per-pre-token cache (labels,
//     currency codes and common words repeat across messages): an open-addressing
//     table over one key arena and one id arena (a lookup hashes the bytes in place:
//     no std::string per pre-token), emptied whole when it fills, so held-out
//     traffic's one-off names and amounts cannot freeze it with stale entries;
//   * truncation to max_body tokens + the <ans> marker, packed as uint16 lengths
//     and int32 ids;
//   * answer decoding: <sep>-split fields, byte-table join, UTF-8 "replace"
//     decode and str.strip(), i.e. exactly ExtractorTokenizer.decode_fields.
//
// Equality with the library is a test (tests/test_fasttok.py: synthetic bodies of
// every family plus random Unicode fuzz).  Plain CPython C API, no third-party code.
#define PY_SSIZE_T_CLEAN
#include <Python.h>

#include <cstdint>
#include <cstring>
#include <string>
#include <algorithm>
#include <utility>
#include <vector>

namespace {

enum : uint8_t { C_L = 1, C_N = 2, C_D = 4, C_S = 8 };

// pre-token bytes -> ids.  One 24-byte slot per entry (hash | 1, key offset / length,
// ids offset / count: a probe touches one cache line); keys and ids live in two arenas.
// Linear probing at <= 50 % load.  Sized for the words that repeat (labels, currency
// codes, common words: a few thousand) so the table stays cache-resident; one-off
// numbers are not cached at all (bpe()).
struct BpeCache {
    static constexpr size_t SLOTS = 1 << 18, MAX_ENTRIES = SLOTS / 2;
    struct Slot {
        uint64_t h;
        uint32_t koff, voff;
        uint16_t klen, vlen;
    };
    std::vector<Slot> slot;
    std::string keys;
    std::vector<int> vals;
    size_t entries = 0;
    BpeCache() : slot(SLOTS, Slot{0, 0, 0, 0, 0}) {}
    static uint64_t hash(const char* s, size_t n) {  // FNV-1a, 64-bit
        uint64_t h = 1469598103934665603ull;
        for (size_t i = 0; i < n; ++i) h = (h ^ (unsigned char)s[i]) * 1099511628211ull;
        return h | 1;
    }
    // ids of the pre-token or nullptr; *at = where it would go
    const int* find(const char* s, size_t n, uint64_t h, size_t* cnt, size_t* at) const {
        for (size_t i = (h >> 7) & (SLOTS - 1);; i = (i + 1) & (SLOTS - 1)) {
            const Slot& e = slot[i];
            if (!e.h) { *at = i; return nullptr; }
            if (e.h == h && e.klen == n && memcmp(keys.data() + e.koff, s, n) == 0) {
                *cnt = e.vlen;
                return vals.data() + e.voff;
            }
        }
    }
    void put(size_t at, const char* s, size_t n, uint64_t h, const int* ids, size_t cnt) {
        if (n > 0xFFFF || cnt > 0xFFFF || keys.size() + n > 0xFFFFFFFFull) return;
        slot[at] = Slot{h, (uint32_t)keys.size(), (uint32_t)vals.size(), (uint16_t)n, (uint16_t)cnt};
        keys.append(s, n);
        vals.insert(vals.end(), ids, ids + cnt);
        ++entries;
    }
    void clear() {
        std::fill(slot.begin(), slot.end(), Slot{0, 0, 0, 0, 0});
        keys.clear();
        vals.clear();
        entries = 0;
    }
};

struct Tok {
    std::vector<std::string> tok_bytes;                       // id -> raw bytes
    void* merge_tab = nullptr;                                 // MergeTable* (defined below)
    int byte_id[256];
    std::vector<uint8_t> cls;                                  // code point -> C_* bits
    std::vector<std::pair<std::string, int>> specials;         // literal -> id
    bool sp_first[256] = {};                                   // first bytes of the specials
    BpeCache cache;
    std::vector<uint32_t> cp, off;                             // scratch of encode_text (GIL held)
    std::vector<int> sym, rk, mid;                             // scratch of bpe()
    std::string buf;
};

inline uint8_t klass(const Tok& t, uint32_t c) { return c < t.cls.size() ? t.cls[c] : 0; }

inline bool is_sym(uint32_t c) {  // $ € £ ₽ ₾ ֏
    return c == 0x24 || c == 0x20AC || c == 0xA3 || c == 0x20BD || c == 0x20BE || c == 0x58F;
}

// ---- pre-tokenizer: one alternative of NUMBER_AWARE_SPLIT at a time, leftmost-first
struct Seg {
    const std::vector<uint32_t>& cp;
    const Tok& t;
    size_t n;
    bool L(size_t i) const { return i < n && (klass(t, cp[i]) & C_L); }
    bool N(size_t i) const { return i < n && (klass(t, cp[i]) & C_N); }
    bool D(size_t i) const { return i < n && (klass(t, cp[i]) & C_D); }
    bool S(size_t i) const { return i < n && (klass(t, cp[i]) & C_S); }
    bool is(size_t i, uint32_t c) const { return i < n && cp[i] == c; }
    size_t run(size_t i, bool (Seg::*f)(size_t) const) const {
        size_t j = i;
        while ((this->*f)(j)) ++j;
        return j - i;
    }
    // \d{1,3}(?:,\d{3})+(?:\.\d+)?  at k (0 = no match)
    size_t grouped(size_t k) const {
        size_t d = run(k, &Seg::D);
        if (d < 1 || d > 3) return 0;  // \d{1,3} must be followed by ','
        size_t p = k + d;
        int groups = 0;
        while (is(p, ',') && D(p + 1) && D(p + 2) && D(p + 3)) {
            p += 4;
            ++groups;
        }
        if (!groups) return 0;
        if (is(p, '.') && D(p + 1)) p += 1 + run(p + 1, &Seg::D);
        return p - k;
    }
    // \d+(?:[.:]\d+)*  at k
    size_t dotted(size_t k) const {
        size_t d = run(k, &Seg::D);
        if (!d) return 0;
        size_t p = k + d;
        while ((is(p, '.') || is(p, ':')) && D(p + 1)) p += 1 + run(p + 1, &Seg::D);
        return p - k;
    }
    bool punct(size_t i) const {  // [^\s\p{L}\p{N}$€£₽₾֏*]
        if (i >= n) return false;
        uint8_t k = klass(t, cp[i]);
        return !(k & (C_S | C_L | C_N)) && !is_sym(cp[i]) && cp[i] != '*';
    }
    bool star(size_t i) const { return is(i, '*'); }
    template <typename F>
    size_t opt_space(size_t i, F f) const {  // " ?X": with the blank first, then without
        if (is(i, ' ')) {
            size_t r = f(i + 1);
            if (r) return r + 1;
        }
        return f(i);
    }
    size_t match(size_t i) const {
        if (is(i, '\'') && i + 1 < n) {  // 's|'t|'re|'ve|'m|'ll|'d
            uint32_t a = cp[i + 1];
            if (a == 's' || a == 't' || a == 'm' || a == 'd') return 2;
            if (i + 2 < n) {
                uint32_t b = cp[i + 2];
                if ((a == 'r' && b == 'e') || (a == 'v' && b == 'e') || (a == 'l' && b == 'l')) return 3;
            }
        }
        size_t r;
        if ((r = opt_space(i, [this](size_t k) { return run(k, &Seg::L); }))) return r;
        if ((r = opt_space(i, [this](size_t k) { return grouped(k); }))) return r;
        if ((r = opt_space(i, [this](size_t k) { return dotted(k); }))) return r;
        if ((r = opt_space(i, [this](size_t k) { return (size_t)(k < n && is_sym(cp[k]) ? 1 : 0); }))) return r;
        if ((r = opt_space(i, [this](size_t k) { return run(k, &Seg::star); }))) return r;
        if ((r = opt_space(i, [this](size_t k) { return run(k, &Seg::punct); }))) return r;
        if (S(i)) {
            size_t w = run(i, &Seg::S);
            if (i + w == n) return w;     // \s+(?!\S) at the end
            if (w >= 2) return w - 1;     // backtrack one: the next char is whitespace
            return w;                     // \s+
        }
        return 0;
    }
};

bool utf8_decode(const char* s, size_t len, std::vector<uint32_t>& cp, std::vector<uint32_t>& off) {
    cp.clear();
    off.clear();
    size_t i = 0;
    while (i < len) {
        unsigned char c = (unsigned char)s[i];
        uint32_t v;
        size_t k;
        if (c < 0x80) { v = c; k = 1; }
        else if ((c >> 5) == 6) { v = c & 0x1F; k = 2; }
        else if ((c >> 4) == 14) { v = c & 0x0F; k = 3; }
        else if ((c >> 3) == 30) { v = c & 0x07; k = 4; }
        else return false;
        if (i + k > len) return false;
        for (size_t j = 1; j < k; ++j) v = (v << 6) | ((unsigned char)s[i + j] & 0x3F);
        cp.push_back(v);
        off.push_back((uint32_t)i);
        i += k;
    }
    off.push_back((uint32_t)len);
    return true;
}

// Merge ranks in an open-addressing table (power-of-two slots, multiplicative hash):
// ~8 k merges fit in L2, one probe per lookup in the common case.
struct MergeTable {
    std::vector<uint64_t> key;   // (a << 32 | b) + 1; 0 = empty
    std::vector<int32_t> rank, id;
    uint64_t mask = 0;
    void init(size_t n) {
        size_t cap = 16;
        while (cap < 2 * n + 16) cap <<= 1;
        key.assign(cap, 0);
        rank.assign(cap, 0);
        id.assign(cap, 0);
        mask = cap - 1;
    }
    static uint64_t h(uint64_t k) { return (k * 0x9E3779B97F4A7C15ull) >> 17; }
    void put(uint64_t k, int r, int m) {
        for (uint64_t i = h(k) & mask;; i = (i + 1) & mask)
            if (!key[i]) { key[i] = k + 1; rank[i] = r; id[i] = m; return; }
    }
    // rank of pair (a, b) or INT32_MAX; its merged id in *m
    int find(int a, int b, int* m) const {
        const uint64_t k = (((uint64_t)(uint32_t)a << 32) | (uint32_t)b) + 1;
        for (uint64_t i = h(k - 1) & mask;; i = (i + 1) & mask) {
            if (key[i] == k) { *m = id[i]; return rank[i]; }
            if (!key[i]) return INT32_MAX;
        }
    }
};

inline const MergeTable& merge_table(const Tok& t) { return *reinterpret_cast<const MergeTable*>(t.merge_tab); }

// a pre-token with more than two ASCII digits is a one-off (an amount, a date, a
// card number): not worth a cache entry, and caching it would evict the words that repeat
inline bool one_off(const char* s, size_t len) {
    int d = 0;
    for (size_t i = 0; i < len; ++i) d += (unsigned)(s[i] - '0') < 10u;
    return d > 2;
}

void bpe(Tok& t, const char* s, size_t len, std::vector<int>& out) {
    const bool cache = !one_off(s, len);
    uint64_t h = 0;
    size_t cnt = 0, slot = 0;
    if (cache) {
        h = BpeCache::hash(s, len);
        if (const int* hit = t.cache.find(s, len, h, &cnt, &slot)) {
            out.insert(out.end(), hit, hit + cnt);
            return;
        }
    }
    const MergeTable& mt = merge_table(t);
    // symbols + the rank / merged id of each adjacent pair, updated locally per merge:
    // O(n) table probes per word instead of O(n^2)
    if (t.sym.size() < len) { t.sym.resize(len); t.rk.resize(len); t.mid.resize(len); }
    int* sym = t.sym.data();
    int* rk = t.rk.data();
    int* mid = t.mid.data();
    for (size_t i = 0; i < len; ++i) sym[i] = t.byte_id[(unsigned char)s[i]];
    size_t n = len;
    for (size_t i = 0; i + 1 < n; ++i) rk[i] = mt.find(sym[i], sym[i + 1], &mid[i]);
    while (n > 1) {
        int best = INT32_MAX;
        size_t bi = 0;
        for (size_t i = 0; i + 1 < n; ++i)
            if (rk[i] < best) { best = rk[i]; bi = i; }
        if (best == INT32_MAX) break;
        // merge the leftmost occurrence of the lowest-rank pair (the library's order: a
        // pair's rank never changes, so its later occurrences are merged next, left to right)
        sym[bi] = mid[bi];
        for (size_t i = bi + 1; i + 1 < n; ++i) { sym[i] = sym[i + 1]; rk[i] = rk[i + 1]; mid[i] = mid[i + 1]; }
        --n;
        if (bi + 1 < n) rk[bi] = mt.find(sym[bi], sym[bi + 1], &mid[bi]);
        else rk[bi] = INT32_MAX;
        if (bi > 0) rk[bi - 1] = mt.find(sym[bi - 1], sym[bi], &mid[bi - 1]);
    }
    if (cache) {
        if (t.cache.entries >= BpeCache::MAX_ENTRIES) {
            t.cache.clear();
            t.cache.find(s, len, h, &cnt, &slot);  // its slot in the emptied table
        }
        t.cache.put(slot, s, len, h, sym, n);
    }
    out.insert(out.end(), sym, sym + n);
}

void encode_text(Tok& t, const char* s, size_t len, std::vector<int>& out) {
    // model_text: the XML line-break entity reaches the model as one "\n"
    std::string& buf = t.buf;
    if (len >= 5 && memmem(s, len, "&#10;", 5)) {
        buf.clear();
        buf.reserve(len);
        for (size_t i = 0; i < len;) {
            if (i + 5 <= len && memcmp(s + i, "&#10;", 5) == 0) {
                buf.push_back('\n');
                i += 5;
            } else {
                buf.push_back(s[i++]);
            }
        }
        s = buf.data();
        len = buf.size();
    }
    std::vector<uint32_t>& cp = t.cp;
    std::vector<uint32_t>& off = t.off;
    size_t pos = 0;
    while (pos <= len) {
        // next special-token literal (leftmost; specials never overlap)
        size_t sp_at = len, sp_len = 0;
        int sp_id = -1;
        for (size_t q = pos; q < len && sp_id < 0; ++q) {
            if (!t.sp_first[(unsigned char)s[q]]) continue;
            for (auto& sp : t.specials)  // list order breaks ties, like the library
                if (sp.first.size() <= len - q && memcmp(s + q, sp.first.data(), sp.first.size()) == 0) {
                    sp_at = q;
                    sp_len = sp.first.size();
                    sp_id = sp.second;
                    break;
                }
        }
        if (sp_at > pos) {
            const char* seg = s + pos;
            size_t seg_len = sp_at - pos;
            if (!utf8_decode(seg, seg_len, cp, off)) {  // not valid UTF-8: bytes as one piece
                bpe(t, seg, seg_len, out);
            } else {
                Seg g{cp, t, cp.size()};
                size_t i = 0, gap = 0;
                while (i < cp.size()) {
                    size_t m = g.match(i);
                    if (!m) { ++i; continue; }
                    if (gap < i) bpe(t, seg + off[gap], off[i] - off[gap], out);
                    bpe(t, seg + off[i], off[i + m] - off[i], out);
                    i += m;
                    gap = i;
                }
                if (gap < cp.size()) bpe(t, seg + off[gap], off[cp.size()] - off[gap], out);
            }
        }
        if (sp_id < 0) break;
        out.push_back(sp_id);
        pos = sp_at + sp_len;
    }
}

const char* CAPSULE = "smsgate._tokfast.Tok";

Tok* get(PyObject* cap) { return (Tok*)PyCapsule_GetPointer(cap, CAPSULE); }

void destroy_tok(Tok* t) {
    delete reinterpret_cast<MergeTable*>(t->merge_tab);
    delete t;
}

void destroy(PyObject* cap) { destroy_tok(get(cap)); }

// new(tok_bytes: list[bytes], merges: list[(a, b, merged)], cls: bytes, specials: list[(bytes, id)])
PyObject* py_new(PyObject*, PyObject* args) {
    PyObject *tb, *mg, *sp;
    Py_buffer cls;
    if (!PyArg_ParseTuple(args, "O!O!y*O!", &PyList_Type, &tb, &PyList_Type, &mg, &cls, &PyList_Type, &sp)) return nullptr;
    Tok* t = new Tok();
    Py_ssize_t V = PyList_GET_SIZE(tb);
    t->tok_bytes.resize(V);
    for (int i = 0; i < 256; ++i) t->byte_id[i] = -1;
    for (Py_ssize_t i = 0; i < V; ++i) {
        PyObject* b = PyList_GET_ITEM(tb, i);
        char* p;
        Py_ssize_t n;
        if (PyBytes_AsStringAndSize(b, &p, &n) < 0) { destroy_tok(t); PyBuffer_Release(&cls); return nullptr; }
        t->tok_bytes[i].assign(p, n);
    }
    MergeTable* mt = new MergeTable();
    t->merge_tab = mt;
    mt->init((size_t)PyList_GET_SIZE(mg));
    for (Py_ssize_t i = 0; i < PyList_GET_SIZE(mg); ++i) {
        int a, b, m;
        if (!PyArg_ParseTuple(PyList_GET_ITEM(mg, i), "iii", &a, &b, &m)) { destroy_tok(t); PyBuffer_Release(&cls); return nullptr; }
        mt->put(((uint64_t)(uint32_t)a << 32) | (uint32_t)b, (int)i, m);
    }
    t->cls.assign((const uint8_t*)cls.buf, (const uint8_t*)cls.buf + cls.len);
    PyBuffer_Release(&cls);
    for (Py_ssize_t i = 0; i < PyList_GET_SIZE(sp); ++i) {
        const char* p;
        Py_ssize_t n;
        int id;
        if (!PyArg_ParseTuple(PyList_GET_ITEM(sp, i), "y#i", &p, &n, &id)) { destroy_tok(t); return nullptr; }
        if (n < 1) { destroy_tok(t); PyErr_SetString(PyExc_ValueError, "empty special token"); return nullptr; }
        t->specials.emplace_back(std::string(p, n), id);
        t->sp_first[(unsigned char)p[0]] = true;
    }
    // single-byte tokens (the byte-level alphabet is always in the vocabulary)
    for (Py_ssize_t i = 0; i < V; ++i)
        if (t->tok_bytes[i].size() == 1) {
            bool special = false;
            for (auto& s : t->specials) special |= (s.second == i);
            if (!special) t->byte_id[(unsigned char)t->tok_bytes[i][0]] = (int)i;
        }
    for (int i = 0; i < 256; ++i)
        if (t->byte_id[i] < 0) { destroy_tok(t); PyErr_Format(PyExc_ValueError, "byte %d has no token", i); return nullptr; }
    return PyCapsule_New(t, CAPSULE, destroy);
}

const char* utf8_of(PyObject* o, Py_ssize_t* n) {
    if (!PyUnicode_Check(o)) { PyErr_SetString(PyExc_TypeError, "expected str"); return nullptr; }
    return PyUnicode_AsUTF8AndSize(o, n);
}

// encode(h, text) -> list[int]
PyObject* py_encode(PyObject*, PyObject* args) {
    PyObject *cap, *text;
    if (!PyArg_ParseTuple(args, "OU", &cap, &text)) return nullptr;
    Tok* t = get(cap);
    if (!t) return nullptr;
    Py_ssize_t n;
    const char* s = utf8_of(text, &n);
    if (!s) return nullptr;
    std::vector<int> ids;
    encode_text(*t, s, (size_t)n, ids);
    PyObject* out = PyList_New((Py_ssize_t)ids.size());
    for (size_t i = 0; i < ids.size(); ++i) PyList_SET_ITEM(out, i, PyLong_FromLong(ids[i]));
    return out;
}

// encode_packed(h, texts: list[str], max_len: int, append_id: int)
//   -> (n_truncated, lens: bytes[uint16 x n], flat: bytes[int32 x sum])
PyObject* py_encode_packed(PyObject*, PyObject* args) {
    PyObject *cap, *texts;
    int max_len, append_id;
    if (!PyArg_ParseTuple(args, "OO!ii", &cap, &PyList_Type, &texts, &max_len, &append_id)) return nullptr;
    Tok* t = get(cap);
    if (!t) return nullptr;
    Py_ssize_t B = PyList_GET_SIZE(texts);
    std::vector<const char*> ptr(B);
    std::vector<Py_ssize_t> len(B);
    std::vector<PyObject*> keep;  // re-encoded texts (lone surrogates -> '?'), released below
    for (Py_ssize_t i = 0; i < B; ++i) {
        PyObject* o = PyList_GET_ITEM(texts, i);
        ptr[i] = utf8_of(o, &len[i]);
        if (!ptr[i]) {
            if (!PyUnicode_Check(o)) return nullptr;
            // a JSON "\udXXX" escape can put a lone surrogate in a body: one bad
            // message must not fail its whole batch
            PyErr_Clear();
            PyObject* b = PyUnicode_AsEncodedString(o, "utf-8", "replace");
            if (!b) { for (auto k : keep) Py_DECREF(k); return nullptr; }
            keep.push_back(b);
            ptr[i] = PyBytes_AS_STRING(b);
            len[i] = PyBytes_GET_SIZE(b);
        }
    }
    std::vector<uint16_t> lens(B);
    std::vector<int32_t> flat;
    flat.reserve((size_t)B * 64);
    long truncated = 0;
    std::vector<int> ids;
    // (the GIL stays held: it is what serialises access to the shared BPE cache)
    for (Py_ssize_t i = 0; i < B; ++i) {
        ids.clear();
        encode_text(*t, ptr[i], (size_t)len[i], ids);
        if (max_len >= 0 && (int)ids.size() > max_len) {
            ids.resize(max_len);
            ++truncated;
        }
        if (append_id >= 0) ids.push_back(append_id);
        lens[i] = (uint16_t)ids.size();
        flat.insert(flat.end(), ids.begin(), ids.end());
    }
    for (auto k : keep) Py_DECREF(k);
    PyObject* l = PyBytes_FromStringAndSize((const char*)lens.data(), (Py_ssize_t)(lens.size() * 2));
    PyObject* f = PyBytes_FromStringAndSize((const char*)flat.data(), (Py_ssize_t)(flat.size() * 4));
    return Py_BuildValue("lNN", truncated, l, f);
}

PyObject* field_str(const std::string& b) {
    PyObject* s = PyUnicode_DecodeUTF8(b.data(), (Py_ssize_t)b.size(), "replace");
    if (!s) return nullptr;
    PyObject* r = PyObject_CallMethod(s, "strip", nullptr);
    Py_DECREF(s);
    return r;
}

// decode_fields(h, buf, offset, n, nfields, sep) -> list[list[str]]
//   buf[offset:] holds lens: uint16[n] then ids: int32[sum(lens)] (serving/protocol.py)
PyObject* py_decode_fields(PyObject*, PyObject* args) {
    PyObject* cap;
    Py_buffer buf;
    Py_ssize_t offset, n;
    int nfields, sep;
    if (!PyArg_ParseTuple(args, "Oy*nnii", &cap, &buf, &offset, &n, &nfields, &sep)) return nullptr;
    Tok* t = get(cap);
    if (!t) { PyBuffer_Release(&buf); return nullptr; }
    const char* base = (const char*)buf.buf + offset;
    Py_ssize_t avail = buf.len - offset;
    if (offset < 0 || n < 0 || avail < 2 * n) {
        PyBuffer_Release(&buf);
        PyErr_SetString(PyExc_ValueError, "decode_fields: truncated buffer");
        return nullptr;
    }
    std::vector<uint16_t> lens(n);
    if (n) memcpy(lens.data(), base, 2 * n);
    size_t total = 0;
    for (auto l : lens) total += l;
    if ((size_t)avail < 2 * (size_t)n + 4 * total) {
        PyBuffer_Release(&buf);
        PyErr_SetString(PyExc_ValueError, "decode_fields: truncated buffer");
        return nullptr;
    }
    const char* ids = base + 2 * n;
    PyObject* out = PyList_New(n);
    size_t p = 0;
    std::string cur;
    const int V = (int)t->tok_bytes.size();
    for (Py_ssize_t r = 0; r < n; ++r) {
        PyObject* row = PyList_New(nfields);
        int k = 0;
        cur.clear();
        bool done = false;
        for (uint16_t j = 0; j < lens[r]; ++j) {
            int32_t tok;
            memcpy(&tok, ids + 4 * (p + j), 4);
            if (done) continue;
            if (tok == sep) {
                PyList_SET_ITEM(row, k++, field_str(cur));
                cur.clear();
                if (k == nfields) done = true;
            } else if (tok >= 0 && tok < V) {
                cur += t->tok_bytes[tok];
            }
        }
        p += lens[r];
        if (k < nfields) PyList_SET_ITEM(row, k++, field_str(cur));
        while (k < nfields) PyList_SET_ITEM(row, k++, PyUnicode_FromStringAndSize("", 0));
        PyList_SET_ITEM(out, r, row);
    }
    PyBuffer_Release(&buf);
    return out;
}

PyObject* py_cache_size(PyObject*, PyObject* args) {
    PyObject* cap;
    if (!PyArg_ParseTuple(args, "O", &cap)) return nullptr;
    Tok* t = get(cap);
    return t ? PyLong_FromSize_t(t->cache.entries) : nullptr;
}

PyMethodDef methods[] = {
    {"new", py_new, METH_VARARGS, "new(tok_bytes, merges, cls, specials) -> handle"},
    {"encode", py_encode, METH_VARARGS, "encode(h, text) -> list[int]"},
    {"encode_packed", py_encode_packed, METH_VARARGS,
     "encode_packed(h, texts, max_len, append_id) -> (n_truncated, lens_u16_bytes, ids_i32_bytes)"},
    {"decode_fields", py_decode_fields, METH_VARARGS,
     "decode_fields(h, buf, offset, n, nfields, sep) -> list[list[str]]"},
    {"cache_size", py_cache_size, METH_VARARGS, "cache_size(h) -> int"},
    {nullptr, nullptr, 0, nullptr}};

PyModuleDef module = {PyModuleDef_HEAD_INIT, "_tokfast", "native BPE encoder / field decoder", -1, methods};

}  // namespace

PyMODINIT_FUNC PyInit__tokfast(void) { return PyModule_Create(&module); }
