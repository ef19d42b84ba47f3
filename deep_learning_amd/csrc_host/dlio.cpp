// dlio — native TFRecord batch reader (include/dlio.h).  Host C++17, built with g++ into
// deep_learning_amd/libdlio.so; replaces utils/data_loader.py:7-40 of the reference
// (TFRecordDataset -> parse(FixedLenFeature) x10 threads -> shuffle -> batch -> repeat).
#include "../../include/dlio.h"

#include <errno.h>
#include <fcntl.h>
#include <nmmintrin.h>
#include <stdarg.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <deque>
#include <memory>
#include <mutex>
#include <random>
#include <string>
#include <thread>
#include <vector>

namespace {

// ------------------------------------------------------------------ CRC-32C
uint32_t g_table[8][256];
bool g_hw = false;

struct CrcInit {
  CrcInit() {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : c >> 1;
      g_table[0][i] = c;
    }
    for (int t = 1; t < 8; ++t)
      for (int i = 0; i < 256; ++i) g_table[t][i] = (g_table[t - 1][i] >> 8) ^ g_table[0][g_table[t - 1][i] & 0xff];
    __builtin_cpu_init();
    g_hw = __builtin_cpu_supports("sse4.2");
  }
} g_crc_init;

__attribute__((target("sse4.2"))) uint32_t crc_hw(const uint8_t* p, size_t n) {
  uint64_t c = 0xFFFFFFFFu;
  while (n >= 8) {
    uint64_t v;
    memcpy(&v, p, 8);
    c = _mm_crc32_u64(c, v);
    p += 8;
    n -= 8;
  }
  uint32_t c32 = (uint32_t)c;
  while (n--) c32 = _mm_crc32_u8(c32, *p++);
  return c32 ^ 0xFFFFFFFFu;
}

uint32_t crc_sw(const uint8_t* p, size_t n) {   // slicing-by-8
  uint32_t c = 0xFFFFFFFFu;
  while (n >= 8) {
    uint32_t lo, hi;
    memcpy(&lo, p, 4);
    memcpy(&hi, p + 4, 4);
    lo ^= c;
    c = g_table[7][lo & 0xff] ^ g_table[6][(lo >> 8) & 0xff] ^ g_table[5][(lo >> 16) & 0xff] ^
        g_table[4][lo >> 24] ^ g_table[3][hi & 0xff] ^ g_table[2][(hi >> 8) & 0xff] ^
        g_table[1][(hi >> 16) & 0xff] ^ g_table[0][hi >> 24];
    p += 8;
    n -= 8;
  }
  while (n--) c = g_table[0][(c ^ *p++) & 0xff] ^ (c >> 8);
  return c ^ 0xFFFFFFFFu;
}

inline uint32_t crc32c(const void* p, size_t n) {
  return g_hw ? crc_hw(static_cast<const uint8_t*>(p), n) : crc_sw(static_cast<const uint8_t*>(p), n);
}
inline uint32_t masked(uint32_t c) { return ((c >> 15) | (c << 17)) + 0xA282EAD8u; }

std::string fmt(const char* f, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, f);
  vsnprintf(buf, sizeof buf, f, ap);
  va_end(ap);
  return buf;
}

thread_local std::string g_open_error;

// ------------------------------------------------------------------ protobuf wire
struct Cursor {
  const uint8_t* p;
  const uint8_t* end;
  bool varint(uint64_t& v) {
    v = 0;
    for (int s = 0; s < 64; s += 7) {
      if (p >= end) return false;
      const uint8_t b = *p++;
      v |= (uint64_t)(b & 0x7f) << s;
      if (!(b & 0x80)) return true;
    }
    return false;
  }
  // next field: number, wire type; for wire 2 the payload span
  bool field(uint32_t& num, uint32_t& wire, Cursor& sub) {
    uint64_t tag;
    if (!varint(tag)) return false;
    num = (uint32_t)(tag >> 3);
    wire = (uint32_t)(tag & 7);
    if (wire == 2) {
      uint64_t n;
      if (!varint(n) || n > (uint64_t)(end - p)) return false;
      sub = Cursor{p, p + n};
      p += n;
    }
    return true;
  }
  bool skip(uint32_t wire) {
    uint64_t v;
    switch (wire) {
      case 0: return varint(v);
      case 1: if (end - p < 8) return false; p += 8; return true;
      case 5: if (end - p < 4) return false; p += 4; return true;
      case 2: return true;   // payload already consumed by field()
      default: return false;
    }
  }
};

struct Feat {
  std::string name;
  int kind;
  int size;
  size_t elem;
};

// ------------------------------------------------------------------ reader
struct Frame {
  const uint8_t* data;
  uint64_t len;
  int32_t file;
};

struct Job {
  int slot;
  int64_t seq;
  std::vector<Frame> frames;
  int next = 0, done = 0;
};

enum SlotState { FREE, FILLING, READY };

struct Reader {
  std::vector<std::string> files;
  std::vector<std::pair<const uint8_t*, size_t>> maps;
  std::vector<Feat> spec;
  int B, repeat, threads, depth;
  int64_t shuffle_buf;
  uint64_t seed;

  std::vector<std::vector<std::vector<uint8_t>>> ring;   // [slot][feature] bytes
  std::vector<SlotState> state;
  std::vector<int64_t> slot_seq;

  std::mutex mu;
  std::condition_variable cv_work, cv_ready, cv_free;
  std::deque<std::unique_ptr<Job>> jobs;
  int64_t produced = 0;          // plans handed to the decoders
  int64_t consumed = 0;          // batches returned by dlio_next
  bool scan_done = false;
  std::atomic<bool> stop{false}, failed{false};   // also read outside the lock by the scanner
  std::string error;
  std::atomic<int64_t> records{0};
  std::thread scanner;
  std::vector<std::thread> workers;

  void fail(const std::string& e) {
    std::lock_guard<std::mutex> g(mu);
    if (!failed) error = e;
    failed = true;
    cv_ready.notify_all();
    cv_work.notify_all();
    cv_free.notify_all();
  }

  // ---------------------------------------------------------------- scanner
  bool emit_plan(std::vector<Frame>& plan) {
    std::unique_lock<std::mutex> g(mu);
    // ring slot for batch `produced` is produced % depth; wait until its previous batch was consumed
    const int slot = (int)(produced % depth);
    cv_free.wait(g, [&] { return stop || failed || state[slot] == FREE; });
    if (stop || failed) return false;
    state[slot] = FILLING;
    auto j = std::make_unique<Job>();
    j->slot = slot;
    j->seq = produced++;
    j->frames.swap(plan);
    jobs.push_back(std::move(j));
    cv_work.notify_all();
    return true;
  }

  void scan() {
    std::mt19937_64 rng(seed);
    std::vector<Frame> buf, plan;
    plan.reserve(B);
    const size_t cap = shuffle_buf > 0 ? (size_t)shuffle_buf : 0;
    auto push = [&](const Frame& f) -> bool {
      plan.push_back(f);
      if ((int)plan.size() == B) {
        if (!emit_plan(plan)) return false;
        plan.clear();
        plan.reserve(B);
      }
      return true;
    };
    auto pick = [&]() {
      const size_t j = (size_t)(((unsigned __int128)rng() * buf.size()) >> 64);
      std::swap(buf[j], buf.back());
      Frame f = buf.back();
      buf.pop_back();
      return f;
    };
    // utils/data_loader.py:30-37 orders the pipeline shuffle -> batch(drop_remainder) -> repeat:
    // every epoch fills and drains its own shuffle buffer and drops its own partial batch, so no
    // batch mixes records of two epochs and each epoch yields floor(records / B) batches.
    for (int ep = 0; ep < repeat; ++ep) {
      for (size_t fi = 0; fi < files.size(); ++fi) {
        const uint8_t* p = maps[fi].first;
        const size_t n = maps[fi].second;
        size_t off = 0;
        while (off < n) {
          if (stop || failed) return;
          if (n - off < 12) return fail(fmt("truncated record header in %s", files[fi].c_str()));
          uint64_t len;
          uint32_t lcrc;
          memcpy(&len, p + off, 8);
          memcpy(&lcrc, p + off + 8, 4);
          if (masked(crc32c(p + off, 8)) != lcrc) return fail(fmt("corrupted record length in %s", files[fi].c_str()));
          if (len > n - off - 12 || n - off - 12 - len < 4) return fail(fmt("truncated record in %s", files[fi].c_str()));
          Frame f{p + off + 12, len, (int32_t)fi};
          off += 12 + len + 4;
          if (cap) {
            buf.push_back(f);
            if (buf.size() >= cap && !push(pick())) return;
          } else if (!push(f)) {
            return;
          }
        }
      }
      while (!buf.empty())               // end of the epoch: drain its shuffle buffer
        if (!push(pick())) return;
      plan.clear();                      // and drop its partial batch (drop_remainder=True)
    }
    std::lock_guard<std::mutex> g(mu);
    scan_done = true;
    cv_ready.notify_all();
  }

  // ---------------------------------------------------------------- decode
  bool decode(const Frame& fr, int slot, int row, std::string& err) {
    uint32_t dcrc;
    memcpy(&dcrc, fr.data + fr.len, 4);
    if (masked(crc32c(fr.data, fr.len)) != dcrc) {
      err = fmt("corrupted record data in %s", files[fr.file].c_str());
      return false;
    }
    const int nf = (int)spec.size();
    int counts[64];
    for (int j = 0; j < nf; ++j) counts[j] = -1;
    Cursor ex{fr.data, fr.data + fr.len};
    uint32_t num, wire;
    Cursor feats{}, entry{}, sub{};
    auto bad = [&]() {
      err = fmt("malformed Example in %s", files[fr.file].c_str());
      return false;
    };
    while (ex.p < ex.end) {
      if (!ex.field(num, wire, feats) || !ex.skip(wire)) return bad();
      if (num != 1 || wire != 2) continue;
      while (feats.p < feats.end) {           // Features.feature map entries
        if (!feats.field(num, wire, entry) || !feats.skip(wire)) return bad();
        if (num != 1 || wire != 2) continue;
        Cursor key{nullptr, nullptr}, val{nullptr, nullptr};
        while (entry.p < entry.end) {
          if (!entry.field(num, wire, sub) || !entry.skip(wire)) return bad();
          if (wire != 2) continue;
          if (num == 1) key = sub;
          else if (num == 2) val = sub;
        }
        if (!key.p) continue;
        const size_t kl = (size_t)(key.end - key.p);
        int j = 0;
        for (; j < nf; ++j)
          if (spec[j].name.size() == kl && memcmp(spec[j].name.data(), key.p, kl) == 0) break;
        if (j == nf) continue;               // a feature outside the spec is ignored
        const Feat& F = spec[j];
        uint8_t* dst = ring[slot][j].data() + (size_t)row * F.size * F.elem;
        int cnt = 0;
        if (val.p) {
          while (val.p < val.end) {          // Feature oneof: 1 bytes, 2 float, 3 int64
            Cursor lst{};
            if (!val.field(num, wire, lst) || !val.skip(wire)) return bad();
            if (wire != 2) continue;
            cnt = 0;
            if ((num == 2 && F.kind != DLIO_FLOAT) || (num == 3 && F.kind != DLIO_INT64) || num == 1) {
              err = fmt("Key: %s. Data types don't match. Expected type: %s", F.name.c_str(),
                        F.kind == DLIO_FLOAT ? "float" : "int64");
              return false;
            }
            while (lst.p < lst.end) {
              Cursor pk{};
              if (!lst.field(num, wire, pk)) return bad();
              if (num != 1) { if (!lst.skip(wire)) return bad(); continue; }
              if (F.kind == DLIO_FLOAT) {
                if (wire == 2) {
                  const size_t nb = (size_t)(pk.end - pk.p);
                  if (nb % 4) return bad();
                  const int nv = (int)(nb / 4);
                  const int w = std::max(0, std::min(nv, F.size - cnt));
                  memcpy(dst + (size_t)cnt * 4, pk.p, (size_t)w * 4);
                  cnt += nv;
                } else if (wire == 5) {
                  if (lst.end - lst.p < 4) return bad();
                  if (cnt < F.size) memcpy(dst + (size_t)cnt * 4, lst.p, 4);
                  lst.p += 4;
                  ++cnt;
                } else {
                  return bad();
                }
              } else {
                uint64_t v;
                if (wire == 2) {
                  while (pk.p < pk.end) {
                    if (!pk.varint(v)) return bad();
                    if (cnt < F.size) memcpy(dst + (size_t)cnt * 8, &v, 8);
                    ++cnt;
                  }
                } else if (wire == 0) {
                  if (!lst.varint(v)) return bad();
                  if (cnt < F.size) memcpy(dst + (size_t)cnt * 8, &v, 8);
                  ++cnt;
                } else {
                  return bad();
                }
              }
            }
          }
        }
        counts[j] = cnt;                     // map semantics: the last entry of a key wins
      }
    }
    for (int j = 0; j < nf; ++j) {
      const int c = counts[j] < 0 ? 0 : counts[j];
      if (c != spec[j].size) {
        err = fmt("Key: %s. Can't parse serialized Example: expected %d values, got %d", spec[j].name.c_str(),
                  spec[j].size, c);
        return false;
      }
    }
    return true;
  }

  void work() {
    constexpr int kChunk = 256;
    std::string err;
    for (;;) {
      Job* job = nullptr;
      int r0 = 0, r1 = 0;
      {
        std::unique_lock<std::mutex> g(mu);
        cv_work.wait(g, [&] {
          if (stop || failed) return true;
          for (auto& j : jobs)
            if (j->next < B) return true;
          return false;
        });
        if (stop || failed) return;
        for (auto& j : jobs)
          if (j->next < B) { job = j.get(); break; }
        r0 = job->next;
        r1 = std::min(B, r0 + kChunk);
        job->next = r1;
      }
      bool ok = true;
      // shuffled frames are scattered over the mapped files: prefetch a few records ahead
      constexpr int kAhead = 6;
      auto prefetch = [&](int r) {
        if (r >= r1) return;
        const Frame& f = job->frames[r];
        for (uint64_t o = 0; o < f.len + 4; o += 64) __builtin_prefetch(f.data + o);
      };
      for (int r = r0; r < r0 + kAhead; ++r) prefetch(r);
      for (int r = r0; r < r1 && ok; ++r) {
        prefetch(r + kAhead);
        ok = decode(job->frames[r], job->slot, r, err);
      }
      if (!ok) return fail(err);
      records.fetch_add(r1 - r0, std::memory_order_relaxed);
      std::lock_guard<std::mutex> g(mu);
      job->done += r1 - r0;
      if (job->done == B) {
        state[job->slot] = READY;
        slot_seq[job->slot] = job->seq;
        for (auto it = jobs.begin(); it != jobs.end(); ++it)
          if (it->get() == job) { jobs.erase(it); break; }
        cv_ready.notify_all();
      }
    }
  }

  int next(void* const* outs) {
    std::unique_lock<std::mutex> g(mu);
    const int slot = (int)(consumed % depth);
    cv_ready.wait(g, [&] {
      return failed || (state[slot] == READY && slot_seq[slot] == consumed) || (scan_done && consumed == produced);
    });
    if (failed) return -1;
    if (state[slot] != READY || slot_seq[slot] != consumed) return 0;
    g.unlock();
    for (size_t j = 0; j < spec.size(); ++j)
      if (!ring[slot][j].empty()) memcpy(outs[j], ring[slot][j].data(), ring[slot][j].size());
    g.lock();
    state[slot] = FREE;
    ++consumed;
    cv_free.notify_all();
    return 1;
  }

  void shutdown() {
    {
      std::lock_guard<std::mutex> g(mu);
      stop = true;
      cv_work.notify_all();
      cv_free.notify_all();
      cv_ready.notify_all();
    }
    if (scanner.joinable()) scanner.join();
    for (auto& t : workers)
      if (t.joinable()) t.join();
    for (auto& m : maps)
      if (m.first && m.second) munmap(const_cast<uint8_t*>(m.first), m.second);
  }
};

}  // namespace

extern "C" void* dlio_open(const char* const* files, int32_t n_files, const dlio_feature* spec, int32_t n_feat,
                           int32_t batch, int32_t repeat, int64_t shuffle_buf, int64_t seed, int32_t threads,
                           int32_t depth) {
  g_open_error.clear();
  if (n_files < 0 || (n_files && !files) || n_feat <= 0 || n_feat > 64 || !spec || batch <= 0 || repeat < 0 ||
      threads <= 0 || depth <= 0) {
    g_open_error = "dlio_open: bad arguments";
    return nullptr;
  }
  auto R = std::make_unique<Reader>();
  R->B = batch;
  R->repeat = repeat;
  R->threads = threads;
  R->depth = depth;
  R->shuffle_buf = shuffle_buf;
  R->seed = seed >= 0 ? (uint64_t)seed : (uint64_t)std::random_device{}() << 32 ^ std::random_device{}();
  for (int j = 0; j < n_feat; ++j) {
    if (!spec[j].name || (spec[j].kind != DLIO_FLOAT && spec[j].kind != DLIO_INT64) || spec[j].size < 0) {
      g_open_error = fmt("dlio_open: bad feature %d", j);
      return nullptr;
    }
    R->spec.push_back({spec[j].name, spec[j].kind, spec[j].size, spec[j].kind == DLIO_FLOAT ? 4u : 8u});
  }
  for (int i = 0; i < n_files; ++i) {
    R->files.emplace_back(files[i]);
    const int fd = open(files[i], O_RDONLY);
    if (fd < 0) {
      g_open_error = fmt("%s: %s", files[i], strerror(errno));
      R->shutdown();
      return nullptr;
    }
    struct stat st;
    fstat(fd, &st);
    const size_t n = (size_t)st.st_size;
    void* p = n ? mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0) : nullptr;
    close(fd);
    if (n && p == MAP_FAILED) {
      g_open_error = fmt("mmap %s: %s", files[i], strerror(errno));
      R->shutdown();
      return nullptr;
    }
    if (n) madvise(p, n, MADV_SEQUENTIAL);
    R->maps.emplace_back(static_cast<const uint8_t*>(p), n);
  }
  R->ring.resize(depth);
  for (auto& s : R->ring)
    for (auto& F : R->spec) s.emplace_back((size_t)batch * F.size * F.elem);
  R->state.assign(depth, FREE);
  R->slot_seq.assign(depth, -1);
  Reader* r = R.get();
  r->scanner = std::thread([r] { r->scan(); });
  for (int t = 0; t < threads; ++t) r->workers.emplace_back([r] { r->work(); });
  return R.release();
}

extern "C" int32_t dlio_next(void* h, void* const* outs) {
  if (!h || !outs) return -2;
  return static_cast<Reader*>(h)->next(outs);
}

extern "C" int64_t dlio_records(void* h) { return h ? static_cast<Reader*>(h)->records.load() : -1; }

extern "C" const char* dlio_last_error(void* h) {
  if (!h) return "NULL handle";
  Reader* r = static_cast<Reader*>(h);
  std::lock_guard<std::mutex> g(r->mu);
  return r->error.c_str();
}

extern "C" const char* dlio_open_error(void) { return g_open_error.c_str(); }

extern "C" void dlio_close(void* h) {
  if (!h) return;
  Reader* r = static_cast<Reader*>(h);
  r->shutdown();
  delete r;
}

extern "C" uint32_t dlio_crc32c(const void* data, int64_t n) { return crc32c(data, (size_t)n); }
extern "C" uint32_t dlio_masked_crc32c(const void* data, int64_t n) { return masked(crc32c(data, (size_t)n)); }
