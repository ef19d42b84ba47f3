// Reference index of one batch: every (sample, slot) table reference sorted by
// row, deduplicated into unique rows with segment offsets and an inverse map.
//
// Uses: (1) a deterministic, atomic-free embedding backward — each unique row's
// gradient is the ordered sum over its segment (replaces the Gather gradient
// UnsortedSegmentSum of deepfm_pipeline.py:188); (2) the row-sharded multi-GPU
// lookup: unique rows grouped by owner rank form the
// all-to-all send lists, the inverse map expands received rows back to slots.
//
// Key of a reference to row r (owner = r % world, local = r / world):
//   (owner << 27) | local     (replicated rows r < replicated_below: owner = world)
// so a sort by key groups rows by owner, then by local row.  References without a key
// (row 0 under the zero-row rule, out-of-range ids) are dropped by the sort's first pass.
//
// The sort is the hand-written stable LSD radix sort of rsort.hip (no library kernels, no
// host synchronisation: the number of valid references stays on the device), so the whole
// index build can run inside a captured hipGraph.
#include "common.h"
#include "rsort.h"
#include <algorithm>

namespace dl {

constexpr int kLocalBits = 27;

// ---------------------------------------------------------------------------
// Segmented unique over the sorted keys in two passes (replaces head flags + a device
// scan + the scatter: three full passes and a decoupled-lookback scan):
//   unique_count_kernel: heads per chunk of kUqChunk sorted keys -> chunk_cnt[c]
//   unique_emit_kernel : one block per chunk; the chunk's exclusive offset is the sum of
//                        the earlier chunks' counts (read from chunk_cnt, summed by the
//                        block — a few thousand ints), then a block scan of the chunk's
//                        head flags gives every element its unique id u, and the same
//                        outputs as before are written (uniq, seg_off, n_uniq, inv,
//                        owner group starts).
constexpr int kUqIpt = 16;                  // keys per thread
constexpr int kUqChunk = 256 * kUqIpt;      // keys per block

__device__ __forceinline__ bool uq_head(const uint32_t* __restrict__ keys, int i, uint32_t k, uint32_t invalid) {
  return k != invalid && (i == 0 || keys[i - 1] != k);
}

__global__ __launch_bounds__(256) void unique_count_kernel(const uint32_t* __restrict__ keys, const int32_t* n_dev,
                                                           int n_max, uint32_t invalid, int32_t* __restrict__ chunk_cnt) {
  const int n = min(*n_dev, n_max);
  const int base = blockIdx.x * kUqChunk;
  int c = 0;
#pragma unroll
  for (int u = 0; u < kUqIpt; ++u) {
    const int i = base + u * 256 + threadIdx.x;   // coalesced: the count does not need the order
    if (i < n) c += uq_head(keys, i, keys[i], invalid) ? 1 : 0;
  }
  c = __reduce_add_sync(~0ull, c);   // wave sum
  __shared__ int ws[4];
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) chunk_cnt[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
}

__global__ __launch_bounds__(256) void unique_emit_kernel(const uint32_t* __restrict__ keys, const int32_t* __restrict__ refs,
                                                          const int32_t* n_dev, int n_max, uint32_t invalid,
                                                          const int32_t* __restrict__ chunk_cnt,
                                                          uint32_t* __restrict__ uniq, int32_t* __restrict__ seg_off,
                                                          int32_t* __restrict__ n_uniq, int32_t* __restrict__ inv,
                                                          int32_t* __restrict__ owner_counts) {
  // Element i = chunk base + r * 256 + tid (round r): every load and every uniq / seg_off
  // store of a round is one coalesced run (a round's heads take consecutive unique ids).
  __shared__ int wsum[4];
  __shared__ int rw[kUqIpt * 4];   // heads per (round, wave), then their exclusive prefix
  __shared__ int base_s;
  const int n = min(*n_dev, n_max);
  if ((long long)blockIdx.x * kUqChunk >= n) return;   // whole block past the valid keys
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int c0 = blockIdx.x * kUqChunk;
  // exclusive offset of this chunk: sum of the earlier chunks' head counts
  int off = 0;
  for (int c = tid; c < (int)blockIdx.x; c += 256) off += chunk_cnt[c];
  off = __reduce_add_sync(~0ull, off);
  if (lane == 0) wsum[wid] = off;
  uint32_t k[kUqIpt];
  int32_t rf[kUqIpt];
  uint64_t hm[kUqIpt];
#pragma unroll
  for (int r = 0; r < kUqIpt; ++r) {
    const int i = c0 + r * 256 + tid;
    k[r] = i < n ? keys[i] : invalid;
    if (inv) rf[r] = i < n ? refs[i] : 0;
  }
#pragma unroll
  for (int r = 0; r < kUqIpt; ++r) {
    const int i = c0 + r * 256 + tid;
    uint32_t pk = __shfl_up(k[r], 1, 64);
    if (lane == 0) pk = i > 0 && i - 1 < n ? keys[i - 1] : invalid;
    const bool hd = i < n && k[r] != invalid && (i == 0 || pk != k[r]);
    hm[r] = __ballot(hd);
    if (lane == 0) rw[r * 4 + wid] = __popcll(hm[r]);
  }
  __syncthreads();
  if (tid < 64) {   // exclusive scan over (round, wave) in element order
    const int x = rw[tid];
    int inc = x;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(inc, o, 64);
      if (lane >= o) inc += y;
    }
    rw[tid] = inc - x;
    if (tid == 0) base_s = wsum[0] + wsum[1] + wsum[2] + wsum[3];
  }
  __syncthreads();
  const int base = base_s;
  const uint64_t le = lane == 63 ? ~0ull : (2ull << lane) - 1;   // lanes <= this one
#pragma unroll
  for (int r = 0; r < kUqIpt; ++r) {
    const int i = c0 + r * 256 + tid;
    const uint32_t kk = k[r];
    const bool valid = i < n && kk != invalid;
    const bool hd = (hm[r] >> lane) & 1;
    const int uu = base + rw[r * 4 + wid] + __popcll(hm[r] & le) - 1;   // heads at or before i, minus one
    uint32_t nk = __shfl_down(kk, 1, 64);
    if (lane == 63) nk = i + 1 < n ? keys[i + 1] : invalid;
    if (hd) {
      uniq[uu] = kk;
      seg_off[uu] = i;
      // first unique row of an owner group (keys sorted by owner): counts follow from the starts
      if (owner_counts) {
        const uint32_t pk = i > 0 ? keys[i - 1] : 0u;
        if (i == 0 || (pk >> kLocalBits) != (kk >> kLocalBits)) owner_counts[kk >> kLocalBits] = uu;
      }
    }
    if (valid && (i + 1 == n || nk == invalid)) {
      seg_off[uu + 1] = i + 1;
      n_uniq[0] = uu + 1;
    }
    if (inv && i < n) inv[rf[r]] = valid ? uu : -1;
  }
}

static void unique_from_sorted(const uint32_t* keys, const int32_t* refs, const int32_t* n_dev, int n_max,
                               uint32_t invalid, int32_t* chunk_cnt, uint32_t* uniq, int32_t* seg_off,
                               int32_t* n_uniq, int32_t* inv, int32_t* owner_counts, hipStream_t s) {
  const int chunks = (n_max + kUqChunk - 1) / kUqChunk;
  hipLaunchKernelGGL(unique_count_kernel, dim3(chunks), dim3(256), 0, s, keys, n_dev, n_max, invalid, chunk_cnt);
  hipLaunchKernelGGL(unique_emit_kernel, dim3(chunks), dim3(256), 0, s, keys, refs, n_dev, n_max, invalid, chunk_cnt,
                     uniq, seg_off, n_uniq, inv, owner_counts);
}

__global__ void index_init_kernel(int32_t* n_uniq, int32_t* seg_off, int32_t* owner_counts, int n_owner) {
  const int t = threadIdx.x;
  if (t == 0) { n_uniq[0] = 0; seg_off[0] = 0; }
  if (owner_counts)
    for (int i = t; i < n_owner; i += blockDim.x) owner_counts[i] = -1;   // group starts, -1 = absent
}

// owner group starts (unique_emit_kernel) -> counts, in owner order.
__global__ void owner_counts_kernel(int32_t* owner_counts, int n_owner, const int32_t* n_uniq) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  int end = n_uniq[0];
  for (int o = n_owner - 1; o >= 0; --o) {
    const int start = owner_counts[o];
    if (start < 0) {
      owner_counts[o] = 0;
    } else {
      owner_counts[o] = end - start;
      end = start;
    }
  }
}

// dl_index_build_pair: the combined index (owner group 0 = the first id set, group 1 = the
// second; owner_counts already turned into counts) split into the two sets' own index arrays:
// the first set's stay in place as a prefix (its n_uniq becomes its own count; its segments,
// inverse entries and sorted references are already right), the second set's are copied out
// with its unique ids, reference numbers and segment offsets rebased to start at 0.
__global__ __launch_bounds__(256) void index_split_kernel(const int32_t* __restrict__ counts, long long n1, long long n2,
                                                          const uint32_t* __restrict__ uniq,
                                                          const int32_t* __restrict__ seg_off,
                                                          const int32_t* __restrict__ refs,
                                                          const int32_t* __restrict__ inv, int32_t* __restrict__ n_uniq,
                                                          uint32_t* __restrict__ uniq2, int32_t* __restrict__ seg2,
                                                          int32_t* __restrict__ refs2, int32_t* __restrict__ n_uniq2,
                                                          int32_t* __restrict__ inv2) {
  const int nt = counts[0], nw = counts[1];
  const int r0 = seg_off[nt];             // the second set's first sorted reference
  const int nr = seg_off[nt + nw] - r0;   // its valid references
  const long long span = max((long long)nw + 1, max((long long)nr, n2));
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < span;
       i += (long long)gridDim.x * blockDim.x) {
    if (i < nw) uniq2[i] = uniq[nt + i] & ((1u << kLocalBits) - 1);
    if (i <= nw) seg2[i] = seg_off[nt + i] - r0;
    if (i < nr) refs2[i] = refs[r0 + i] - (int32_t)n1;
    if (i < n2) {
      const int u = inv[n1 + i];
      inv2[i] = u >= 0 ? u - nt : -1;
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    n_uniq[0] = nt;
    n_uniq2[0] = nw;
  }
}

static size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// workspace: the sort's, then the unique step's per-chunk head counts and the valid count
struct IndexWs {
  void* sort;
  size_t sort_bytes;
  int32_t* chunk_cnt;
  int32_t* n_valid;
  int32_t* pair_counts;   // dl_index_build_pair: the two id sets' unique counts
};

static IndexWs carve(void* ws, int64_t n) {
  char* p = reinterpret_cast<char*>(ws);
  IndexWs w;
  w.sort = p;
  w.sort_bytes = rsort_workspace_bytes(n);
  p += align256(w.sort_bytes);
  w.chunk_cnt = reinterpret_cast<int32_t*>(p);
  p += align256((size_t)((n + kUqChunk - 1) / kUqChunk + 1) * 4);
  w.n_valid = reinterpret_cast<int32_t*>(p);
  w.pair_counts = w.n_valid + 4;
  return w;
}

// Bits of the compressed key range (rsort.h): owner-major, lrange rows per owner.
static int compressed_bits(int64_t n_rows, int world, int rep_below, uint32_t& lrange) {
  lrange = (uint32_t)((n_rows + world - 1) / world);
  const uint64_t max_excl = rep_below > 0 ? (uint64_t)world * lrange + (uint64_t)rep_below : (uint64_t)world * lrange;
  int b = 1;
  while (b < 32 && (1ull << b) < max_excl) ++b;
  return b;
}

__global__ void batch_err_reset_kernel(int32_t* err) { err[0] = 0; }

// The batch's ids against the rows they address (the checks the forward kernels make, done
// before the step begins): single cate column c < S reads deep row id + deep_cate_offset and,
// with FM, FM row id + fm_cate_offset; multi-hot columns read row id + deep_cate_offset; wide
// ids address wdl_weights rows [0, wide_rows).
__global__ __launch_bounds__(256) void validate_batch_kernel(dl_emb_layout L, const int64_t* __restrict__ cate,
                                                             const int64_t* __restrict__ wide, int wide_cols,
                                                             int wide_ld, int64_t wide_rows,
                                                             int32_t* __restrict__ err) {
  const long long nc = cate ? (long long)L.batch * L.cate_ld : 0;
  const long long nw = wide ? (long long)L.batch * wide_cols : 0;
  bool bad = false;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < nc + nw;
       i += (long long)gridDim.x * blockDim.x) {
    if (i < nc) {
      const int c = (int)(i % L.cate_ld);
      const int64_t id = cate[i];
      const int64_t d = id + L.deep_cate_offset;
      bad |= d < 0 || d >= L.n_rows;
      if (c < L.cate_fields && L.use_fm) {
        const int64_t f = id + L.fm_cate_offset;
        bad |= f < 0 || f >= L.n_rows;
      }
    } else {
      const long long k = i - nc;
      const int64_t id = wide[(k / wide_cols) * wide_ld + k % wide_cols];
      bad |= id < 0 || id >= wide_rows;
    }
  }
  if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(err, DL_STATUS_BAD_ID);
}

}  // namespace dl

using namespace dl;

extern "C" int dl_validate_batch(const dl_emb_layout* L, const int64_t* cate, const int64_t* wide, int32_t wide_cols,
                                 int32_t wide_ld, int64_t wide_rows, int32_t reset, int32_t* err, void* stream) {
  DL_CHECK_ARG(L && err, "NULL argument");
  DL_CHECK_ARG(!wide || (wide_cols > 0 && wide_ld >= wide_cols && wide_rows > 0), "bad wide shape");
  DL_CHECK_ARG(!cate || L->cate_ld > 0, "bad cate shape");
  hipStream_t s = as_stream(stream);
  if (reset) hipLaunchKernelGGL(batch_err_reset_kernel, dim3(1), dim3(1), 0, s, err);
  const long long n = (cate ? (long long)L->batch * L->cate_ld : 0) + (wide ? (long long)L->batch * wide_cols : 0);
  if (n > 0) {
    long long blocks = (n + 255) / 256;
    if (blocks > 2048) blocks = 2048;
    hipLaunchKernelGGL(validate_batch_kernel, dim3((unsigned)blocks), dim3(256), 0, s, *L, cate, wide, wide_cols,
                       wide_ld, wide_rows, err);
  }
  DL_RETURN_LAUNCH("dl_validate_batch");
}

extern "C" int64_t dl_index_workspace_bytes(int64_t n_refs) {
  if (n_refs <= 0 || n_refs > (1LL << 30)) return -1;
  return (int64_t)(align256(rsort_workspace_bytes(n_refs)) + align256((size_t)((n_refs + kUqChunk - 1) / kUqChunk + 1) * 4) +
                   256);
}

extern "C" int dl_index_build(const dl_emb_layout* L, const int64_t* cate, int32_t world,
                              int32_t replicated_below, void* ws, int64_t ws_bytes,
                              uint32_t* sorted_keys, int32_t* sorted_refs, uint32_t* uniq_keys,
                              int32_t* seg_off, int32_t* n_uniq, int32_t* inv, int32_t* owner_counts,
                              int32_t* err, void* stream) {
  DL_CHECK_ARG(L && cate && ws && sorted_keys && sorted_refs && uniq_keys && seg_off && n_uniq, "NULL argument");
  DL_CHECK_ARG(world >= 1 && world < 32, "world %d out of range", world);
  DL_CHECK_ARG(L->n_rows / world < (1LL << kLocalBits), "too many rows per shard for the 27-bit local key");
  DL_CHECK_ARG(replicated_below >= 0 && replicated_below < (1 << kLocalBits), "bad replicated_below");
  const long long n_ll = (long long)L->batch * index_slots(*L);
  DL_CHECK_ARG(n_ll < (1LL << 30), "too many references");
  const int n = (int)n_ll;
  DL_CHECK_ARG(ws_bytes >= dl_index_workspace_bytes(n > 0 ? n : 1), "workspace too small");
  hipStream_t s = as_stream(stream);
  // zeroing by a kernel (not a memset node): keeps every node of a captured step a kernel
  hipLaunchKernelGGL(index_init_kernel, dim3(1), dim3(64), 0, s, n_uniq, seg_off, owner_counts, world + 1);
  if (n == 0) return 0;
  IndexWs w = carve(ws, n);
  uint32_t lrange;
  const int bits = compressed_bits(L->n_rows, world, replicated_below, lrange);
  RsSource src{};
  src.kind = 1;
  src.L = *L;
  src.cate = cate;
  src.world = world;
  src.rep_below = replicated_below;
  src.err = err;
  src.inv = inv;
  if (int rc = rsort_pairs(src, n, lrange, bits, w.sort, w.sort_bytes, sorted_keys, sorted_refs, w.n_valid, s)) {
    set_error("dl_index_build: radix sort failed (%d)", rc);
    return 2;
  }
  unique_from_sorted(sorted_keys, sorted_refs, w.n_valid, n, 0xFFFFFFFFu, w.chunk_cnt, uniq_keys, seg_off, n_uniq, inv,
                     owner_counts, s);
  if (owner_counts)
    hipLaunchKernelGGL(owner_counts_kernel, dim3(1), dim3(64), 0, s, owner_counts, world + 1, n_uniq);
  DL_RETURN_LAUNCH("dl_index_build");
}

extern "C" int dl_index_build_pair(const dl_emb_layout* L, const int64_t* cate, const dl_emb_layout* L2,
                                   const int64_t* cate2, void* ws, int64_t ws_bytes, uint32_t* sorted_keys,
                                   int32_t* sorted_refs, uint32_t* uniq_keys, int32_t* seg_off, int32_t* n_uniq,
                                   int32_t* inv, uint32_t* uniq2, int32_t* sorted_refs2, int32_t* seg_off2,
                                   int32_t* n_uniq2, int32_t* inv2, int32_t* err, void* stream) {
  DL_CHECK_ARG(L && cate && L2 && cate2 && ws && sorted_keys && sorted_refs && uniq_keys && seg_off && n_uniq && inv &&
                   uniq2 && sorted_refs2 && seg_off2 && n_uniq2 && inv2,
               "NULL argument");
  DL_CHECK_ARG(L->n_rows < (1LL << kLocalBits) && L2->n_rows < (1LL << kLocalBits), "too many rows for the 27-bit key");
  const long long n1 = (long long)L->batch * index_slots(*L), n2 = (long long)L2->batch * index_slots(*L2);
  DL_CHECK_ARG(n1 > 0 && n2 > 0 && n1 + n2 < (1LL << 30), "bad reference counts");
  const int n = (int)(n1 + n2);
  DL_CHECK_ARG(ws_bytes >= dl_index_workspace_bytes(n), "workspace too small");
  hipStream_t s = as_stream(stream);
  IndexWs w = carve(ws, n);
  hipLaunchKernelGGL(index_init_kernel, dim3(1), dim3(64), 0, s, n_uniq, seg_off, w.pair_counts, 2);
  // owner-major compressed keys: group 0 = [0, lrange), group 1 = [lrange, 2 lrange)
  const uint32_t lrange = (uint32_t)std::max(L->n_rows, L2->n_rows);
  int bits = 1;
  while (bits < 32 && (1ull << bits) < 2ull * lrange) ++bits;
  RsSource src{};
  src.kind = 1;
  src.L = *L;
  src.cate = cate;
  src.world = 1;
  src.rep_below = 0;
  src.err = err;
  src.inv = inv;
  src.n1 = n1;
  src.L2 = *L2;
  src.cate2 = cate2;
  if (int rc = rsort_pairs(src, n, lrange, bits, w.sort, w.sort_bytes, sorted_keys, sorted_refs, w.n_valid, s)) {
    set_error("dl_index_build_pair: radix sort failed (%d)", rc);
    return 2;
  }
  unique_from_sorted(sorted_keys, sorted_refs, w.n_valid, n, 0xFFFFFFFFu, w.chunk_cnt, uniq_keys, seg_off, n_uniq, inv,
                     w.pair_counts, s);
  hipLaunchKernelGGL(owner_counts_kernel, dim3(1), dim3(64), 0, s, w.pair_counts, 2, n_uniq);
  long long g = (std::max(n1, n2) + 255) / 256;
  if (g > 4096) g = 4096;
  hipLaunchKernelGGL(index_split_kernel, dim3((unsigned)g), dim3(256), 0, s, w.pair_counts, n1, n2, uniq_keys, seg_off,
                     sorted_refs, inv, n_uniq, uniq2, seg_off2, sorted_refs2, n_uniq2, inv2);
  DL_RETURN_LAUNCH("dl_index_build_pair");
}

extern "C" int dl_sort_unique(const int32_t* keys, int64_t n_keys, int32_t key_bits, void* ws, int64_t ws_bytes,
                              int32_t* sorted_keys, int32_t* sorted_pos, int32_t* uniq_keys, int32_t* seg_off,
                              int32_t* n_uniq, int32_t* inv, void* stream) {
  DL_CHECK_ARG(keys && ws && sorted_keys && sorted_pos && uniq_keys && seg_off && n_uniq, "NULL argument");
  DL_CHECK_ARG(key_bits >= 1 && key_bits <= 31, "key_bits %d out of range", key_bits);
  DL_CHECK_ARG(n_keys >= 0 && n_keys < (1LL << 30), "bad n_keys");
  const int n = (int)n_keys;
  DL_CHECK_ARG(ws_bytes >= dl_index_workspace_bytes(n > 0 ? n : 1), "workspace too small");
  hipStream_t s = as_stream(stream);
  hipLaunchKernelGGL(index_init_kernel, dim3(1), dim3(64), 0, s, n_uniq, seg_off, (int32_t*)nullptr, 0);
  if (n == 0) return 0;
  IndexWs w = carve(ws, n);
  RsSource src{};
  src.kind = 0;
  src.keys = reinterpret_cast<const uint32_t*>(keys);
  if (int rc = rsort_pairs(src, n, 0u, key_bits, w.sort, w.sort_bytes, reinterpret_cast<uint32_t*>(sorted_keys),
                           sorted_pos, w.n_valid, s)) {
    set_error("dl_sort_unique: radix sort failed (%d)", rc);
    return 2;
  }
  // keys are non-negative (< 2^key_bits): never equal to the 0xFFFFFFFF marker
  unique_from_sorted(reinterpret_cast<const uint32_t*>(sorted_keys), sorted_pos, w.n_valid, n, 0xFFFFFFFFu,
                     w.chunk_cnt, reinterpret_cast<uint32_t*>(uniq_keys), seg_off, n_uniq, inv, (int32_t*)nullptr, s);
  DL_RETURN_LAUNCH("dl_sort_unique");
}
