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
// so a sort by key groups rows by owner, then by local row.  Invalid refs
// (row 0 under the zero-row rule, out-of-range ids) get key 0xFFFFFFFF and sort last.
#include <hipcub/hipcub.hpp>

#include "common.h"

namespace dl {

constexpr int kLocalBits = 27;

__device__ __forceinline__ bool row_ok_i(int64_t row, int zero_row0) {
  return row > 0 || (row == 0 && !zero_row0);
}

__global__ __launch_bounds__(256) void make_refs_kernel(dl_emb_layout L, const int64_t* __restrict__ cate, int world,
                                                        int rep_below, uint32_t kInvalidKey,
                                                        uint32_t* __restrict__ keys,
                                                        int32_t* __restrict__ refs, int32_t* err) {
  const int S = L.cate_fields;
  const int ns = index_slots(L);
  const long long n = (long long)L.batch * ns;
  for (long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (long long)gridDim.x * blockDim.x) {
    const int b = (int)(k / ns), s = (int)(k % ns);
    int64_t row;
    const int mb = index_multi_base(L);
    if (L.use_fm && s < S) row = cate[(long long)b * L.cate_ld + s] + L.fm_cate_offset;
    else if (s < mb) row = cate[(long long)b * L.cate_ld + (L.use_fm ? s - S : s)] + L.deep_cate_offset;
    else row = cate[(long long)b * L.cate_ld + S + (s - mb)] + L.deep_cate_offset;   // multi-hot id
    uint32_t key = kInvalidKey;
    if (row < 0 || row >= L.n_rows) {
      if (err) atomicOr(err, 1);
    } else if (row_ok_i(row, L.zero_row0)) {
      if (row < rep_below) key = ((uint32_t)world << kLocalBits) | (uint32_t)row;
      else key = ((uint32_t)(row % world) << kLocalBits) | (uint32_t)(row / world);
    }
    keys[k] = key;
    refs[k] = (int32_t)k;
  }
}

// Multi-hot batches are mostly padding (id 0 -> invalid key): the valid (key, ref) pairs are
// compacted in ref order before the sort, and inv starts at -1 for every reference.
__global__ __launch_bounds__(256) void valid_flags_kernel(const uint32_t* __restrict__ keys, int n, uint32_t kInvalidKey,
                                                          int32_t* __restrict__ flags, int32_t* __restrict__ inv) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    flags[i] = keys[i] != kInvalidKey ? 1 : 0;
    if (inv) inv[i] = -1;
  }
}

__global__ __launch_bounds__(256) void compact_kernel(const uint32_t* __restrict__ keys, const int32_t* __restrict__ pos1,
                                                      int n, uint32_t kInvalidKey, uint32_t* __restrict__ kout,
                                                      int32_t* __restrict__ rout, int32_t* __restrict__ n_valid) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    if (keys[i] != kInvalidKey) {
      const int p = pos1[i] - 1;
      kout[p] = keys[i];
      rout[p] = i;
    }
    if (i + 1 == n) n_valid[0] = pos1[i];
  }
}

__global__ __launch_bounds__(256) void head_flags_kernel(const uint32_t* __restrict__ keys, int n, uint32_t kInvalidKey,
                                                         int32_t* __restrict__ flags) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint32_t k = keys[i];
    flags[i] = (k != kInvalidKey && (i == 0 || keys[i - 1] != k)) ? 1 : 0;
  }
}

__global__ __launch_bounds__(256) void scatter_index_kernel(const uint32_t* __restrict__ keys, const int32_t* __restrict__ refs,
                                                            const int32_t* __restrict__ uid1, int n, int world,
                                                            uint32_t kInvalidKey,
                                                            uint32_t* __restrict__ uniq, int32_t* __restrict__ seg_off,
                                                            int32_t* __restrict__ n_uniq, int32_t* __restrict__ inv,
                                                            int32_t* __restrict__ owner_counts) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint32_t k = keys[i];
    if (k == kInvalidKey) {
      if (inv) inv[refs[i]] = -1;
      continue;
    }
    const int u = uid1[i] - 1;
    const bool head = (i == 0 || keys[i - 1] != k);
    if (head) {
      uniq[u] = k;
      seg_off[u] = i;
      // first unique row of an owner group (keys are sorted by owner): its start index.
      // Counts follow from the starts (owner_counts_kernel) — no per-row atomics on the
      // world+1 counters, which serialised 3.2 M updates (38 ms at one rank).
      if (owner_counts && (i == 0 || (keys[i - 1] >> kLocalBits) != (k >> kLocalBits)))
        owner_counts[k >> kLocalBits] = u;
    }
    if (i + 1 == n || keys[i + 1] == kInvalidKey) {
      seg_off[u + 1] = i + 1;
      n_uniq[0] = u + 1;
    }
    if (inv) inv[refs[i]] = u;
  }
}

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

__global__ __launch_bounds__(256) void unique_count_kernel(const uint32_t* __restrict__ keys, int n, uint32_t invalid,
                                                           int32_t* __restrict__ chunk_cnt) {
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
                                                          int n, uint32_t invalid, const int32_t* __restrict__ chunk_cnt,
                                                          uint32_t* __restrict__ uniq, int32_t* __restrict__ seg_off,
                                                          int32_t* __restrict__ n_uniq, int32_t* __restrict__ inv,
                                                          int32_t* __restrict__ owner_counts) {
  __shared__ int wsum[4];
  __shared__ int base_s;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  // exclusive offset of this chunk: sum of the earlier chunks' head counts
  int off = 0;
  for (int c = tid; c < (int)blockIdx.x; c += 256) off += chunk_cnt[c];
  off = __reduce_add_sync(~0ull, off);
  if (lane == 0) wsum[wid] = off;
  __syncthreads();
  if (tid == 0) base_s = wsum[0] + wsum[1] + wsum[2] + wsum[3];
  __syncthreads();
  const int base = base_s;
  // this thread's kUqIpt consecutive keys
  const int i0 = blockIdx.x * kUqChunk + tid * kUqIpt;
  uint32_t k[kUqIpt];
  int h = 0;
  uint32_t prev = (i0 > 0 && i0 - 1 < n) ? keys[i0 - 1] : 0u;
  if (i0 + kUqIpt <= n) {   // 64-B aligned run: four 16-B loads
#pragma unroll
    for (int q = 0; q < kUqIpt / 4; ++q) {
      const uint4 v = reinterpret_cast<const uint4*>(keys + i0)[q];
      k[4 * q] = v.x; k[4 * q + 1] = v.y; k[4 * q + 2] = v.z; k[4 * q + 3] = v.w;
    }
  } else {
#pragma unroll
    for (int u = 0; u < kUqIpt; ++u) k[u] = i0 + u < n ? keys[i0 + u] : invalid;
  }
#pragma unroll
  for (int u = 0; u < kUqIpt; ++u) {
    const int i = i0 + u;
    const bool hd = i < n && k[u] != invalid && (i == 0 || (u == 0 ? prev : k[u - 1]) != k[u]);
    h += hd ? 1 : 0;
  }
  // block exclusive scan of the per-thread head counts (wave scan + wave totals)
  int x = h;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  __syncthreads();
  if (lane == 63) wsum[wid] = x;
  __syncthreads();
  int wbase = 0;
  for (int w = 0; w < wid; ++w) wbase += wsum[w];
  int run = base + wbase + x - h;   // heads before this thread's first key
  // the key after this thread's run and the refs of the run (16-B loads when whole);
  // the loop below is fully unrolled (no break/continue: k[] stays in registers)
  const uint32_t after = i0 + kUqIpt < n ? keys[i0 + kUqIpt] : invalid;
  int32_t rf[kUqIpt];
  if (inv) {
    if (i0 + kUqIpt <= n) {
#pragma unroll
      for (int q = 0; q < kUqIpt / 4; ++q) {
        const int4 v = reinterpret_cast<const int4*>(refs + i0)[q];
        rf[4 * q] = v.x; rf[4 * q + 1] = v.y; rf[4 * q + 2] = v.z; rf[4 * q + 3] = v.w;
      }
    } else {
#pragma unroll
      for (int u = 0; u < kUqIpt; ++u) rf[u] = i0 + u < n ? refs[i0 + u] : 0;
    }
  }
#pragma unroll
  for (int u = 0; u < kUqIpt; ++u) {
    const int i = i0 + u;
    const uint32_t kk = k[u];
    const uint32_t pk = u == 0 ? prev : k[u - 1];
    const uint32_t nk = u + 1 < kUqIpt ? k[u + 1] : after;
    const bool valid = i < n && kk != invalid;
    const bool hd = valid && (i == 0 || pk != kk);
    run += hd ? 1 : 0;
    const int uu = run - 1;
    if (hd) {
      uniq[uu] = kk;
      seg_off[uu] = i;
      // first unique row of an owner group (keys sorted by owner): counts follow from the starts
      if (owner_counts && (i == 0 || (pk >> kLocalBits) != (kk >> kLocalBits))) owner_counts[kk >> kLocalBits] = uu;
    }
    if (valid && (i + 1 == n || nk == invalid)) {
      seg_off[uu + 1] = i + 1;
      n_uniq[0] = uu + 1;
    }
    if (inv && i < n) inv[rf[u]] = valid ? uu : -1;
  }
}

static void unique_from_sorted(const uint32_t* keys, const int32_t* refs, int n, uint32_t invalid, int32_t* chunk_cnt,
                               uint32_t* uniq, int32_t* seg_off, int32_t* n_uniq, int32_t* inv,
                               int32_t* owner_counts, hipStream_t s) {
  const int chunks = (n + kUqChunk - 1) / kUqChunk;
  hipLaunchKernelGGL(unique_count_kernel, dim3(chunks), dim3(256), 0, s, keys, n, invalid, chunk_cnt);
  hipLaunchKernelGGL(unique_emit_kernel, dim3(chunks), dim3(256), 0, s, keys, refs, n, invalid, chunk_cnt, uniq,
                     seg_off, n_uniq, inv, owner_counts);
}

// copies the compacted pairs back into the sort's input arrays
__global__ __launch_bounds__(256) void iota_refs_copy_kernel(const uint32_t* __restrict__ kin, const int32_t* __restrict__ rin,
                                                             int n, uint32_t* __restrict__ kout, int32_t* __restrict__ rout) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    kout[i] = kin[i];
    rout[i] = rin[i];
  }
}

__global__ void index_init_kernel(int32_t* n_uniq, int32_t* seg_off, int32_t* owner_counts, int n_owner) {
  const int t = threadIdx.x;
  if (t == 0) { n_uniq[0] = 0; seg_off[0] = 0; }
  if (owner_counts)
    for (int i = t; i < n_owner; i += blockDim.x) owner_counts[i] = -1;   // group starts, -1 = absent
}

// owner group starts (scatter_index_kernel) -> counts, in owner order.
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

struct IndexWs {
  uint32_t* keys_in;
  int32_t* refs_in;
  int32_t* flags;
  int32_t* uid1;
  void* temp;
  size_t temp_bytes;
};

static size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// Onesweep radix sort over the key's significant bits only (25 for a 26M-row table).
// (11-bit digits would save a pass, but rocPRIM's match-rank variant that fits them
// in LDS ran 3x slower on gfx950 — measured; the default 8-bit digits stay.)
static hipError_t sort_pairs(void* temp, size_t& bytes, const uint32_t* kin, uint32_t* kout, const int32_t* vin,
                             int32_t* vout, int n, int end_bit, hipStream_t s) {
  return hipcub::DeviceRadixSort::SortPairs(temp, bytes, kin, kout, vin, vout, n, 0, end_bit, s);
}

static size_t cub_temp_bytes(int n) {
  size_t a = 0, b = 0;
  sort_pairs(nullptr, a, nullptr, nullptr, nullptr, nullptr, n, 32, 0);
  hipcub::DeviceScan::InclusiveSum(nullptr, b, (int32_t*)nullptr, (int32_t*)nullptr, n);
  return a > b ? a : b;
}

// Bits of the sorted key range: keys are < 2^end_bit, the all-ones value marks invalid refs.
static int key_bits(int64_t n_rows, int world, int rep_below) {
  uint64_t max_key;
  if (world == 1 && rep_below == 0) max_key = (uint64_t)n_rows;            // row; n_rows itself = headroom
  else max_key = ((uint64_t)(rep_below > 0 ? world : world - 1) << kLocalBits) | ((1u << kLocalBits) - 1);
  int b = 1;
  while (b < 32 && (max_key + 1) > (1ull << b) - 1) ++b;
  return b;
}

static IndexWs carve(void* ws, int n) {
  char* p = reinterpret_cast<char*>(ws);
  IndexWs w;
  w.keys_in = reinterpret_cast<uint32_t*>(p); p += align256((size_t)n * 4);
  w.refs_in = reinterpret_cast<int32_t*>(p); p += align256((size_t)n * 4);
  w.flags = reinterpret_cast<int32_t*>(p); p += align256((size_t)n * 4);
  w.uid1 = reinterpret_cast<int32_t*>(p); p += align256((size_t)n * 4);
  w.temp = p;
  w.temp_bytes = cub_temp_bytes(n);
  return w;
}

}  // namespace dl

using namespace dl;

extern "C" int64_t dl_index_workspace_bytes(int64_t n_refs) {
  if (n_refs <= 0 || n_refs > (1LL << 30)) return -1;
  const int n = (int)n_refs;
  return (int64_t)(4 * align256((size_t)n * 4) + align256(cub_temp_bytes(n)));
}

extern "C" int dl_index_build(const dl_emb_layout* L, const int64_t* cate, int32_t world,
                              int32_t replicated_below, void* ws, int64_t ws_bytes,
                              uint32_t* sorted_keys, int32_t* sorted_refs, uint32_t* uniq_keys,
                              int32_t* seg_off, int32_t* n_uniq, int32_t* inv, int32_t* owner_counts,
                              int32_t* err, void* stream) {
  DL_CHECK_ARG(L && cate && ws && sorted_keys && sorted_refs && uniq_keys && seg_off && n_uniq, "NULL argument");
  DL_CHECK_ARG(world >= 1 && world < 32, "world %d out of range", world);
  DL_CHECK_ARG(L->n_rows / world < (1LL << kLocalBits), "too many rows per shard for the 27-bit local key");
  const int S = L->cate_fields;
  const long long n_ll = (long long)L->batch * index_slots(*L);
  DL_CHECK_ARG(n_ll < (1LL << 30), "too many references");
  int n = (int)n_ll;
  DL_CHECK_ARG(ws_bytes >= dl_index_workspace_bytes(n > 0 ? n : 1), "workspace too small");
  hipStream_t s = as_stream(stream);
  // zeroing by a kernel (not a memset node): keeps every node of a captured step a kernel
  hipLaunchKernelGGL(index_init_kernel, dim3(1), dim3(64), 0, s, n_uniq, seg_off, owner_counts, world + 1);
  if (n == 0) return 0;
  IndexWs w = carve(ws, n);
  const int grid = (int)((n + 255) / 256 < 8192 ? (n + 255) / 256 : 8192);
  const int end_bit = key_bits(L->n_rows, world, replicated_below);
  const uint32_t invalid = end_bit >= 32 ? 0xFFFFFFFFu : (uint32_t)((1ull << end_bit) - 1);
  hipLaunchKernelGGL(make_refs_kernel, dim3(grid), dim3(256), 0, s, *L, cate, world, replicated_below, invalid,
                     w.keys_in, w.refs_in, err);
  size_t tb = w.temp_bytes;
  const uint32_t* sort_keys = w.keys_in;
  const int32_t* sort_refs = w.refs_in;
  int ns_sort = n;
  if (L->multi_width > 0) {
    // compact the valid references (ref order kept), then sort only those; the sorted
    // arrays hold them first.  One stream sync to learn the count (the sort's size).
    hipLaunchKernelGGL(valid_flags_kernel, dim3(grid), dim3(256), 0, s, w.keys_in, n, invalid, w.flags, inv);
    if (hipcub::DeviceScan::InclusiveSum(w.temp, tb, w.flags, w.uid1, n, s) != hipSuccess) {
      set_error("dl_index_build: scan failed");
      return 3;
    }
    // compacted pairs go to the sorted_* arrays (free until the sort), then sort into place
    uint32_t* ck = reinterpret_cast<uint32_t*>(w.flags);   // flags are consumed by the scan
    hipLaunchKernelGGL(compact_kernel, dim3(grid), dim3(256), 0, s, w.keys_in, w.uid1, n, invalid, ck, sorted_refs,
                       n_uniq);
    int32_t nv = 0;
    if (hipMemcpyAsync(&nv, n_uniq, sizeof(int32_t), hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess) {
      set_error("dl_index_build: count readback failed");
      return 4;
    }
    hipLaunchKernelGGL(iota_refs_copy_kernel, dim3(grid), dim3(256), 0, s, ck, sorted_refs, nv, w.keys_in, w.refs_in);
    hipLaunchKernelGGL(index_init_kernel, dim3(1), dim3(64), 0, s, n_uniq, seg_off, owner_counts, world + 1);
    ns_sort = nv;
    tb = w.temp_bytes;
  }
  if (ns_sort > 0 &&
      sort_pairs(w.temp, tb, sort_keys, sorted_keys, sort_refs, sorted_refs, ns_sort, end_bit, s) != hipSuccess) {
    set_error("dl_index_build: radix sort failed");
    return 2;
  }
  n = ns_sort;
  if (n == 0) DL_RETURN_LAUNCH("dl_index_build");
  unique_from_sorted(sorted_keys, sorted_refs, n, invalid, w.flags, uniq_keys, seg_off, n_uniq, inv, owner_counts, s);
  if (owner_counts)
    hipLaunchKernelGGL(owner_counts_kernel, dim3(1), dim3(64), 0, s, owner_counts, world + 1, n_uniq);
  DL_RETURN_LAUNCH("dl_index_build");
}

namespace dl {
__global__ __launch_bounds__(256) void iota_copy_kernel(const int32_t* __restrict__ keys, int n, int32_t* __restrict__ kout,
                                                        int32_t* __restrict__ pos) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    kout[i] = keys[i];
    pos[i] = i;
  }
}
}  // namespace dl

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
  const int grid = (int)((n + 255) / 256 < 8192 ? (n + 255) / 256 : 8192);
  const uint32_t invalid = 0xFFFFFFFFu;   // keys are non-negative (< 2^key_bits): never equal
  hipLaunchKernelGGL(iota_copy_kernel, dim3(grid), dim3(256), 0, s, keys, n, (int32_t*)w.keys_in, w.refs_in);
  size_t tb = w.temp_bytes;
  if (sort_pairs(w.temp, tb, w.keys_in, (uint32_t*)sorted_keys, w.refs_in, sorted_pos, n, key_bits, s) !=
      hipSuccess) {
    set_error("dl_sort_unique: radix sort failed");
    return 2;
  }
  unique_from_sorted((const uint32_t*)sorted_keys, sorted_pos, n, invalid, w.flags, (uint32_t*)uniq_keys, seg_off,
                     n_uniq, inv, (int32_t*)nullptr, s);
  DL_RETURN_LAUNCH("dl_sort_unique");
}
