// Native decoder of the load-style batches (include/dlio.h, dlio_unpickle_batch).
//
// The reference's load-style models train from a list of pickled batch dicts
// (utils/data_loader_load.py:128-136 pickles {"labels", "cont_feats", "cate_feats", ...} per
// batch; models/wdl.py:296 unpickles one per step).  pickle.loads builds Python objects under
// the GIL and copies every array once more before the host-to-device transfer; this decoder
// walks the pickle opcodes itself and writes each requested field straight into the caller's
// (pinned) buffer, converted to float32 or int64, with no Python object built and no GIL held
// (ctypes releases it), so a worker thread can decode the next batch beside the training loop.
//
// It reads protocols 3-5 as pickle.dumps writes them for a dict whose values are numpy arrays
// (numpy's _reconstruct + __setstate__ form, protocols 3-4; _frombuffer, protocol 5 in-band)
// or nested lists of numbers (the reference's own lists of lists).  It constructs nothing: the
// only globals it accepts are those data descriptions (numpy's reconstructors, ndarray, dtype),
// anything else — another global, an object array, an out-of-band buffer — returns 1 and the
// caller falls back to pickle.loads.
#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "dlio.h"

namespace {

enum Kind { K_NONE, K_BOOL, K_INT, K_FLOAT, K_STR, K_BYTES, K_SEQ, K_DICT, K_GLOBAL, K_DTYPE, K_ARRAY, K_RECON };
enum Glob { G_OTHER, G_RECONSTRUCT, G_NDARRAY, G_DTYPE, G_FROMBUFFER };

struct Val {
  Kind k = K_NONE;
  int64_t i = 0;                 // int / bool
  double f = 0;                  // float
  const uint8_t* p = nullptr;    // str / bytes payload (a view into the pickle)
  int64_t n = 0;                 // its length
  std::vector<int> items;        // sequence items, or dict key, value pairs
  Glob g = G_OTHER;              // global
  char dk = 0;                   // dtype kind ('f', 'i', 'u', 'b') and item size
  int isz = 0;
  bool big = false;              // dtype byte order '>'
  int dt = -1;                   // array: its dtype value
  std::vector<int64_t> shape;    // array shape
  bool fortran = false;
};

constexpr int kMark = -1;

struct Parser {
  const uint8_t* d;
  int64_t n, pos = 0;
  std::vector<Val> vals;
  std::vector<int> stack, memo;
  int status = 0;   // 0 ok, 1 unsupported form, -1 malformed

  Parser(const uint8_t* data, int64_t len) : d(data), n(len) { vals.reserve(1024); }

  bool need(int64_t k) {   // k more bytes at pos; k from an 8-byte length may be near INT64_MAX
    if (k < 0 || k > n - pos) { status = -1; return false; }
    return true;
  }
  uint64_t rd(int k) {   // little-endian unsigned
    uint64_t x = 0;
    for (int j = 0; j < k; ++j) x |= (uint64_t)d[pos + j] << (8 * j);
    pos += k;
    return x;
  }
  int add(Val v) {
    vals.push_back(std::move(v));
    return (int)vals.size() - 1;
  }
  int pop() {
    if (stack.empty() || stack.back() == kMark) { status = -1; return 0; }
    const int x = stack.back();
    stack.pop_back();
    return x;
  }
  std::vector<int> pop_mark() {
    std::vector<int> out;
    while (!stack.empty() && stack.back() != kMark) {
      out.push_back(stack.back());
      stack.pop_back();
    }
    if (stack.empty()) { status = -1; return out; }
    stack.pop_back();
    return std::vector<int>(out.rbegin(), out.rend());
  }
  bool str_is(const Val& v, const char* s) const {
    return v.k == K_STR && (int64_t)strlen(s) == v.n && memcmp(v.p, s, v.n) == 0;
  }
  static Glob classify(const std::string& mod, const std::string& name) {
    const bool np_core = mod == "numpy.core.multiarray" || mod == "numpy._core.multiarray";
    const bool np_num = mod == "numpy.core.numeric" || mod == "numpy._core.numeric";
    if (np_core && name == "_reconstruct") return G_RECONSTRUCT;
    if (np_num && name == "_frombuffer") return G_FROMBUFFER;
    if (mod == "numpy" && name == "ndarray") return G_NDARRAY;
    if (mod == "numpy" && name == "dtype") return G_DTYPE;
    return G_OTHER;
  }
  bool shape_of(int t, std::vector<int64_t>& shape) {
    const Val& s = vals[t];
    if (s.k != K_SEQ) return false;
    shape.clear();
    for (int it : s.items) {
      if (vals[it].k != K_INT) return false;
      shape.push_back(vals[it].i);
    }
    return true;
  }
  void unsupported() { if (status == 0) status = 1; }

  void reduce() {
    const int args = pop(), fn = pop();
    if (status) return;
    const Val& F = vals[fn];
    const Val& A = vals[args];
    if (F.k != K_GLOBAL || A.k != K_SEQ) return unsupported();
    if (F.g == G_RECONSTRUCT) {   // _reconstruct(ndarray, (0,), b'b'): the array BUILD fills in
      Val r;
      r.k = K_RECON;
      stack.push_back(add(r));
    } else if (F.g == G_DTYPE) {  // dtype('f4', False, True)
      if (A.items.empty() || vals[A.items[0]].k != K_STR) return unsupported();
      const Val& s = vals[A.items[0]];
      if (s.n < 2 || s.n > 3) return unsupported();
      Val t;
      t.k = K_DTYPE;
      t.dk = (char)s.p[0];
      t.isz = atoi(std::string((const char*)s.p + 1, s.n - 1).c_str());
      if (!strchr("fiub", t.dk) || !(t.isz == 1 || t.isz == 2 || t.isz == 4 || t.isz == 8)) return unsupported();
      stack.push_back(add(t));
    } else if (F.g == G_FROMBUFFER) {   // _frombuffer(buffer, dtype, shape, order)
      if (A.items.size() != 4) return unsupported();
      const Val& b = vals[A.items[0]];
      if (b.k != K_BYTES || vals[A.items[1]].k != K_DTYPE) return unsupported();
      Val a;
      a.k = K_ARRAY;
      a.p = b.p;
      a.n = b.n;
      a.dt = A.items[1];
      if (!shape_of(A.items[2], a.shape)) return unsupported();
      a.fortran = str_is(vals[A.items[3]], "F");
      stack.push_back(add(a));
    } else {
      return unsupported();
    }
  }

  void build() {
    const int st = pop();
    if (status) return;
    if (stack.empty() || stack.back() == kMark) { status = -1; return; }
    Val& o = vals[stack.back()];
    const Val& S = vals[st];
    if (o.k == K_DTYPE) {   // (3, '<', None, None, None, -1, -1, 0)
      if (S.k != K_SEQ || S.items.size() < 2) return unsupported();
      const Val& bo = vals[S.items[1]];
      if (str_is(bo, ">")) o.big = true;
      else if (!str_is(bo, "<") && !str_is(bo, "|") && !str_is(bo, "=")) return unsupported();
      if (S.items.size() >= 4 && vals[S.items[3]].k != K_NONE) return unsupported();   // structured
      return;
    }
    if (o.k == K_RECON) {   // (1, shape, dtype, is_fortran, raw bytes)
      if (S.k != K_SEQ || S.items.size() != 5) return unsupported();
      std::vector<int64_t> shape;
      if (!shape_of(S.items[1], shape) || vals[S.items[2]].k != K_DTYPE) return unsupported();
      const Val& raw = vals[S.items[4]];
      if (raw.k != K_BYTES) return unsupported();   // an object array pickles a list here
      o.k = K_ARRAY;
      o.shape = shape;
      o.dt = S.items[2];
      o.fortran = vals[S.items[3]].k == K_BOOL && vals[S.items[3]].i;
      o.p = raw.p;
      o.n = raw.n;
      return;
    }
    unsupported();
  }

  int run() {
    while (status == 0) {
      if (!need(1)) break;
      const uint8_t op = d[pos++];
      switch (op) {
        case 0x80: if (need(1)) pos += 1; break;                      // PROTO
        case 0x95: if (need(8)) pos += 8; break;                      // FRAME
        case '.': { const int r = pop(); return status ? -1 : r; }    // STOP
        case '(': stack.push_back(kMark); break;                      // MARK
        case '}': { Val v; v.k = K_DICT; stack.push_back(add(v)); break; }
        case ']': case ')': { Val v; v.k = K_SEQ; stack.push_back(add(v)); break; }
        case 0x94:                                                    // MEMOIZE
          if (stack.empty() || stack.back() == kMark) { status = -1; break; }
          memo.push_back(stack.back());
          break;
        case 'q': case 'r': {                                         // BINPUT, LONG_BINPUT
          const int w = op == 'q' ? 1 : 4;
          if (!need(w)) break;
          const uint64_t idx = rd(w);
          if (stack.empty() || stack.back() == kMark || idx > (1u << 24)) { status = -1; break; }
          if (memo.size() <= idx) memo.resize(idx + 1, kMark);
          memo[idx] = stack.back();
          break;
        }
        case 'h': case 'j': {                                         // BINGET, LONG_BINGET
          const int w = op == 'h' ? 1 : 4;
          if (!need(w)) break;
          const uint64_t idx = rd(w);
          if (idx >= memo.size() || memo[idx] == kMark) { status = -1; break; }
          stack.push_back(memo[idx]);
          break;
        }
        case 0x8c: case 'X': case 0x8d:                               // str
        case 'C': case 'B': case 0x8e: case 0x96: {                   // bytes, bytearray
          const int w = (op == 0x8c || op == 'C') ? 1 : (op == 'X' || op == 'B') ? 4 : 8;
          if (!need(w)) break;
          const int64_t len = (int64_t)rd(w);
          if (len < 0 || !need(len)) { status = -1; break; }
          Val v;
          v.k = (op == 0x8c || op == 'X' || op == 0x8d) ? K_STR : K_BYTES;
          v.p = d + pos;
          v.n = len;
          pos += len;
          stack.push_back(add(v));
          break;
        }
        case 0x98: break;                                             // READONLY_BUFFER
        case 0x97: unsupported(); break;                              // NEXT_BUFFER (out of band)
        case 'J': case 'K': case 'M': {                               // BININT, BININT1, BININT2
          const int w = op == 'J' ? 4 : op == 'K' ? 1 : 2;
          if (!need(w)) break;
          Val v;
          v.k = K_INT;
          v.i = op == 'J' ? (int64_t)(int32_t)rd(4) : (int64_t)rd(w);
          stack.push_back(add(v));
          break;
        }
        case 0x8a: {                                                  // LONG1
          if (!need(1)) break;
          const int len = d[pos++];
          if (len > 8) { unsupported(); break; }
          if (!need(len)) break;
          uint64_t x = len ? rd(len) : 0;
          if (len && len < 8 && (x >> (8 * len - 1)) & 1) x |= ~0ull << (8 * len);   // sign
          Val v;
          v.k = K_INT;
          v.i = (int64_t)x;
          stack.push_back(add(v));
          break;
        }
        case 'G': {                                                   // BINFLOAT (big-endian)
          if (!need(8)) break;
          uint64_t x = 0;
          for (int j = 0; j < 8; ++j) x = (x << 8) | d[pos + j];
          pos += 8;
          Val v;
          v.k = K_FLOAT;
          memcpy(&v.f, &x, 8);
          stack.push_back(add(v));
          break;
        }
        case 0x88: case 0x89: { Val v; v.k = K_BOOL; v.i = op == 0x88; stack.push_back(add(v)); break; }
        case 'N': { Val v; stack.push_back(add(v)); break; }
        case 't': { Val v; v.k = K_SEQ; v.items = pop_mark(); stack.push_back(add(v)); break; }
        case 0x85: case 0x86: case 0x87: {                            // TUPLE1..3
          const int m = op - 0x84;
          Val v;
          v.k = K_SEQ;
          v.items.resize(m);
          for (int j = m - 1; j >= 0; --j) v.items[j] = pop();
          stack.push_back(add(v));
          break;
        }
        case 'a': {                                                   // APPEND
          const int x = pop();
          if (status || stack.empty() || stack.back() == kMark || vals[stack.back()].k != K_SEQ) { status = -1; break; }
          vals[stack.back()].items.push_back(x);
          break;
        }
        case 'e': {                                                   // APPENDS
          std::vector<int> xs = pop_mark();
          if (status || stack.empty() || stack.back() == kMark || vals[stack.back()].k != K_SEQ) { status = -1; break; }
          auto& it = vals[stack.back()].items;
          it.insert(it.end(), xs.begin(), xs.end());
          break;
        }
        case 's': {                                                   // SETITEM
          const int v = pop(), k = pop();
          if (status || stack.empty() || stack.back() == kMark || vals[stack.back()].k != K_DICT) { status = -1; break; }
          vals[stack.back()].items.push_back(k);
          vals[stack.back()].items.push_back(v);
          break;
        }
        case 'u': {                                                   // SETITEMS
          std::vector<int> xs = pop_mark();
          if (status || (xs.size() & 1) || stack.empty() || stack.back() == kMark || vals[stack.back()].k != K_DICT) {
            status = -1;
            break;
          }
          auto& it = vals[stack.back()].items;
          it.insert(it.end(), xs.begin(), xs.end());
          break;
        }
        case 'c': {                                                   // GLOBAL "module\nname\n"
          const uint8_t* e1 = (const uint8_t*)memchr(d + pos, '\n', n - pos);
          if (!e1) { status = -1; break; }
          const std::string mod((const char*)d + pos, e1 - (d + pos));
          pos = e1 - d + 1;
          const uint8_t* e2 = (const uint8_t*)memchr(d + pos, '\n', n - pos);
          if (!e2) { status = -1; break; }
          const std::string name((const char*)d + pos, e2 - (d + pos));
          pos = e2 - d + 1;
          Val v;
          v.k = K_GLOBAL;
          v.g = classify(mod, name);
          stack.push_back(add(v));
          break;
        }
        case 0x93: {                                                  // STACK_GLOBAL
          const int nm = pop(), md = pop();
          if (status) break;
          if (vals[nm].k != K_STR || vals[md].k != K_STR) { status = -1; break; }
          Val v;
          v.k = K_GLOBAL;
          v.g = classify(std::string((const char*)vals[md].p, vals[md].n), std::string((const char*)vals[nm].p, vals[nm].n));
          stack.push_back(add(v));
          break;
        }
        case 'R': reduce(); break;                                    // REDUCE
        case 'b': build(); break;                                     // BUILD
        default: unsupported(); break;
      }
    }
    return -1;
  }
};

template <typename T>
inline T num_of(const Val& v) {
  return v.k == K_FLOAT ? (T)v.f : (T)v.i;
}

template <typename T>
inline T elem(const uint8_t* p, char dk, int isz) {
  switch (dk) {
    case 'f': {
      if (isz == 4) { float x; memcpy(&x, p, 4); return (T)x; }
      if (isz == 8) { double x; memcpy(&x, p, 8); return (T)x; }
      return (T)0;   // float16: rejected before
    }
    case 'i':
      if (isz == 1) return (T)(int8_t)p[0];
      if (isz == 2) { int16_t x; memcpy(&x, p, 2); return (T)x; }
      if (isz == 4) { int32_t x; memcpy(&x, p, 4); return (T)x; }
      { int64_t x; memcpy(&x, p, 8); return (T)x; }
    default:   // 'u', 'b'
      if (isz == 1) return (T)p[0];
      if (isz == 2) { uint16_t x; memcpy(&x, p, 2); return (T)x; }
      if (isz == 4) { uint32_t x; memcpy(&x, p, 4); return (T)x; }
      { uint64_t x; memcpy(&x, p, 8); return (T)x; }
  }
}

// One field's rows before any copy: rows, or -2 unsupported / -3 shape mismatch.  (A list's
// rows are checked as they are copied: fill.)
int64_t check(const Parser& P, int vi, int32_t size, int64_t cap_rows) {
  const Val& v = P.vals[vi];
  if (v.k == K_ARRAY) {
    const Val& t = P.vals[v.dt];
    if (t.big || (t.dk == 'f' && t.isz == 2)) return -2;
    int64_t rows = v.shape.empty() ? 1 : v.shape[0], cols = 1;
    for (size_t j = 1; j < v.shape.size(); ++j) cols *= v.shape[j];
    if (v.fortran && v.shape.size() > 1 && rows > 1 && cols > 1) return -2;
    if (cols != size || rows > cap_rows || rows < 0) return -3;
    if (v.n != rows * cols * t.isz) return -3;
    return rows;
  }
  if (v.k == K_SEQ) {   // a list of rows: each a list / tuple of numbers, or a number (size 1)
    const int64_t rows = (int64_t)v.items.size();
    return rows > cap_rows ? -3 : rows;
  }
  return -2;
}

// Rows [r0, r1) of a checked field into out (rows x size of T): 0, or -2 / -3 for a list row
// of another form.  Row ranges are disjoint pieces of out, so ranges can run on any threads.
template <typename T>
int fill(const Parser& P, int vi, int32_t size, T* out, char want_dk, int64_t r0, int64_t r1) {
  const Val& v = P.vals[vi];
  if (v.k == K_ARRAY) {
    const Val& t = P.vals[v.dt];
    const int64_t j0 = r0 * size, j1 = r1 * size;
    if (t.dk == want_dk && t.isz == (int)sizeof(T))
      memcpy(out + j0, v.p + j0 * (int64_t)sizeof(T), (size_t)(j1 - j0) * sizeof(T));
    else
      for (int64_t j = j0; j < j1; ++j) out[j] = elem<T>(v.p + j * t.isz, t.dk, t.isz);
    return 0;
  }
  for (int64_t r = r0; r < r1; ++r) {
    const Val& row = P.vals[v.items[r]];
    if (row.k == K_SEQ) {
      if ((int64_t)row.items.size() != size) return -3;
      for (int32_t c = 0; c < size; ++c) {
        const Val& x = P.vals[row.items[c]];
        if (x.k != K_INT && x.k != K_FLOAT && x.k != K_BOOL) return -2;
        out[r * size + c] = num_of<T>(x);
      }
    } else if (row.k == K_INT || row.k == K_FLOAT || row.k == K_BOOL) {
      if (size != 1) return -3;
      out[r] = num_of<T>(row);
    } else {
      return -2;
    }
  }
  return 0;
}

// Threads one decode may use for its copies (DLIO_DECODE_THREADS, default 4).  A C5 batch is
// 31 MB: on the GPU box a worker's decode took 1.80-2.25 ms on one thread, 1.43-1.44 ms on 4 and
// 1.46-1.65 ms on 8, the drop-in step the same 2.2 ms throughout (profiles/r05bg/) — the feed
// is bound by the host's memory traffic (two workers' copies beside the staging DMA).
int decode_threads() {
  static const int n = [] {
    const char* e = getenv("DLIO_DECODE_THREADS");
    const int v = e ? atoi(e) : 4;
    return v < 1 ? 1 : (v > 64 ? 64 : v);
  }();
  return n;
}

}  // namespace

extern "C" int32_t dlio_unpickle_batch(const void* data, int64_t n, const dlio_feature* fields, int32_t n_fields,
                                       int64_t cap_rows, void* const* outs, int64_t* rows_out) {
  if (!data || n <= 0 || (n_fields > 0 && (!fields || !outs)) || !rows_out) return -1;
  Parser P(reinterpret_cast<const uint8_t*>(data), n);
  const int root = P.run();
  if (P.status > 0) return 1;
  if (P.status < 0 || root < 0 || P.vals[root].k != K_DICT) return P.status < 0 ? -1 : 1;
  const Val& D = P.vals[root];
  std::vector<int> vis(n_fields, -1);
  for (int32_t f = 0; f < n_fields; ++f) {
    for (size_t j = 0; j + 1 < D.items.size(); j += 2)
      if (P.str_is(P.vals[D.items[j]], fields[f].name)) vis[f] = D.items[j + 1];
    if (vis[f] < 0) return 1;   // a missing key: pickle.loads and the model's own KeyError
  }
  // every field checked first; then the copies / conversions as row pieces of at least 1 MB
  // (once the batch is large: 4 MB or more), the pieces dealt to a team of threads
  std::vector<int64_t> rs(n_fields, -2);
  for (int32_t f = 0; f < n_fields; ++f) {
    rs[f] = check(P, vis[f], fields[f].size, cap_rows);
    if (rs[f] < 0) return 1;    // unsupported form or shape: the Python path decides (and raises)
  }
  struct Piece { int32_t f; int64_t r0, r1; };
  std::vector<Piece> pieces;
  const int nt = n >= (4 << 20) ? decode_threads() : 1;
  int64_t total = 0;
  for (int32_t f = 0; f < n_fields; ++f) total += rs[f] * (int64_t)fields[f].size * 8;
  const int64_t piece_bytes = nt > 1 ? std::max<int64_t>(1 << 20, total / (2 * nt)) : INT64_MAX;
  for (int32_t f = 0; f < n_fields; ++f) {
    const int64_t row_bytes = std::max<int64_t>(1, (int64_t)fields[f].size * 8);
    const int64_t step = std::max<int64_t>(1, piece_bytes / row_bytes);
    for (int64_t r = 0; r < rs[f]; r += step) pieces.push_back({f, r, std::min(rs[f], r + step)});
  }
  std::vector<int> st(pieces.size(), 0);
  std::atomic<size_t> next{0};
  auto work = [&]() {
    for (size_t i; (i = next.fetch_add(1)) < pieces.size();) {
      const Piece& q = pieces[i];
      st[i] = fields[q.f].kind == DLIO_FLOAT
                  ? fill<float>(P, vis[q.f], fields[q.f].size, reinterpret_cast<float*>(outs[q.f]), 'f', q.r0, q.r1)
                  : fill<int64_t>(P, vis[q.f], fields[q.f].size, reinterpret_cast<int64_t*>(outs[q.f]), 'i', q.r0,
                                  q.r1);
    }
  };
  const int helpers = (int)std::min<size_t>((size_t)nt, pieces.size()) - 1;
  std::vector<std::thread> th;
  for (int i = 0; i < helpers; ++i) th.emplace_back(work);
  work();
  for (auto& t : th) t.join();
  for (int v : st)
    if (v < 0) return 1;
  int64_t rows = -1;
  for (int32_t f = 0; f < n_fields; ++f) {
    if (rows >= 0 && rs[f] != rows) return 1;
    rows = rs[f];
  }
  *rows_out = rows < 0 ? 0 : rows;
  return 0;
}
