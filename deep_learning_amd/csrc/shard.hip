// Row-sharded embedding tables across GPUs: owner-side
// gather / scatter-add of exchanged rows and the dense-gradient slab reducer.
//
// Row r of the logical table lives on rank r % world at local row r / world
// (cyclic: Zipf-hot low ids spread over all ranks); rows below `replicated`
// (the deepfm_pipeline cont-field rows hit by every sample) are replicated and
// their gradients all-reduced with the dense parameters.
#include "common.h"

namespace dl {

// out[i] = table[ids[i]] (E floats), out1[i] = first[ids[i]]; E/4 lanes per row.  An id of -1
// (an empty slot of a fixed-capacity exchange block) gives a zero row.
__global__ __launch_bounds__(256) void shard_gather_kernel(const float4* __restrict__ table, const float* __restrict__ first,
                                                           const int32_t* __restrict__ ids, long long n, int lpr,
                                                           float4* __restrict__ out, float* __restrict__ out1) {
  const long long total = n * lpr;
  for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (long long)gridDim.x * blockDim.x) {
    const long long i = t / lpr;
    const int q = (int)(t % lpr);
    const int r = ids[i];
    out[t] = r >= 0 ? table[(long long)r * lpr + q] : make_float4(0.f, 0.f, 0.f, 0.f);
    if (first && q == 0) out1[i] = r >= 0 ? first[r] : 0.f;
  }
}

// G[ids[i]] += g[i], G1[ids[i]] += g1[i]; duplicates across peers -> f32 atomics (ids < 0: empty slots).
__global__ __launch_bounds__(256) void shard_scatter_kernel(const float* __restrict__ g, const float* __restrict__ g1,
                                                            const int32_t* __restrict__ ids, long long n, int E,
                                                            float* __restrict__ G, float* __restrict__ G1,
                                                            uint8_t* __restrict__ touched) {
  const long long total = n * E;
  for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (long long)gridDim.x * blockDim.x) {
    const long long i = t / E;
    const int d = (int)(t % E);
    const int r = ids[i];
    if (r < 0) continue;
    atomicAdd(G + (long long)r * E + d, g[t]);
    if (d == 0) {
      if (g1 && G1) atomicAdd(G1 + r, g1[i]);
      touched[r] = 1;
    }
  }
}

// out[i] = sum_s slab[s*stride + i]
__global__ __launch_bounds__(256) void slab_sum_kernel(const float* __restrict__ slab, int nslab, long long stride,
                                                       long long n, float* __restrict__ out) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    float g = 0.f;
    for (int s = 0; s < nslab; ++s) g += slab[s * stride + i];
    out[i] = g;
  }
}

// few elements, many slabs (the head's per-block partials): one wave per element
__global__ __launch_bounds__(256) void slab_sum_wave_kernel(const float* __restrict__ slab, int nslab, long long stride,
                                                            long long n, float* __restrict__ out) {
  const long long i = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (i >= n) return;
  float g = 0.f;
  for (int s = lane; s < nslab; s += 64) g += slab[s * stride + i];
  g = wave_sum(g);
  if (lane == 0) out[i] = g;
}

// local row of each unique key (key & (2^27-1)); the send list of the id exchange
__global__ void keys_to_local_kernel(const uint32_t* __restrict__ keys, const int32_t* __restrict__ n_uniq,
                                     long long cap, int32_t* __restrict__ out) {
  const long long nu = n_uniq[0];
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < nu && i < cap;
       i += (long long)gridDim.x * blockDim.x)
    out[i] = (int32_t)(keys[i] & ((1u << 27) - 1));
}

// ---------------------------------------------------------------------------
// Row-sharded wdl_weights (wdl.py:241-285; the wide / deep cross-logit weights, sharded like
// the table: row r on rank r % world at local row r / world).
__global__ __launch_bounds__(256) void shard_gather_scalar_kernel(const float* __restrict__ w,
                                                                  const int32_t* __restrict__ ids, long long n,
                                                                  float* __restrict__ out) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const int r = ids[i];
    out[i] = r >= 0 ? w[r] : 0.f;
  }
}

// Arrived per-row wide gradients (int64 fixed point, the sender's segment sums) added to the
// owner's gradient: integer atomics, so the sum does not depend on arrival order.
__global__ __launch_bounds__(256) void shard_add_fixed_kernel(const int64_t* __restrict__ g,
                                                              const int32_t* __restrict__ ids, long long n,
                                                              int64_t* __restrict__ G, uint8_t* __restrict__ touched) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const int r = ids[i];
    if (r < 0) continue;
    atomicAdd(reinterpret_cast<unsigned long long*>(G + r), (unsigned long long)g[i]);
    if (touched) touched[r] = 1;
  }
}

// The deep-output rows row0 + j (j < H; the all-reduced batch sums of dz*h) that this rank owns,
// folded into its fixed-point gradient.
__global__ void wide_fold_owned_kernel(const float* __restrict__ gdeep, int H, long long row0, int world, int rank,
                                       int64_t* __restrict__ G, uint8_t* __restrict__ touched) {
  for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < H; j += gridDim.x * blockDim.x) {
    const long long r = row0 + j;
    if (r % world != rank) continue;
    const long long lr = r / world;
    atomicAdd(reinterpret_cast<unsigned long long*>(G + lr), (unsigned long long)wide_fixed(gdeep[j]));
    if (touched) touched[lr] = 1;
  }
}

// out[j] = this rank's value of row row0 + j if it owns it, else 0 (summed over ranks: the
// replicated copy of the deep-output rows every rank's cross logit reads).
__global__ void wide_owned_values_kernel(const float* __restrict__ w, int H, long long row0, int world, int rank,
                                         float* __restrict__ out) {
  for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < H; j += gridDim.x * blockDim.x) {
    const long long r = row0 + j;
    out[j] = (r % world == rank) ? w[r / world] : 0.f;
  }
}

// ids of the local wide table: out[k] = offset + inv[k] (-1 for a reference without a row)
__global__ __launch_bounds__(256) void wide_local_ids_kernel(const int32_t* __restrict__ inv, long long n,
                                                             long long offset, int64_t* __restrict__ out) {
  for (long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (long long)gridDim.x * blockDim.x) {
    const int u = inv[k];
    out[k] = u < 0 ? -1 : offset + u;
  }
}

// ---------------------------------------------------------------------------
// Fixed-capacity exchange blocks (SURVEY.md §8(e) steps 3-5 and the gradient return, as one
// captured graph: every message size is fixed when the step is captured, the true counts travel
// in a header beside the data).  A rank's exchange arrays hold 2W - 1 blocks of `cap` slots:
//   blocks [0, W)      owner side: block p = what peer p sends this rank (block `rank` is this
//                      rank's own requests, written in place — never sent);
//   blocks [W, 2W - 1) sender side: the requests to (and the answers from) each other peer p,
//                      block W + p - (p > rank).
// shard_block(p) is where this rank's slots for owner p live; the replicated rows (owner W,
// deepfm_pipeline's FM cont-field rows referenced by cate ids) follow all blocks.
__device__ __forceinline__ long long shard_block(int p, int world, int rank) {
  return p == rank ? p : world + p - (p > rank ? 1 : 0);
}

struct RouteArgs {
  const uint32_t* uniq;      // the batch index's unique keys, grouped by owner (dl_index_build)
  const int32_t* n_uniq;
  const int32_t* counts;     // [W + 1] unique rows per owner (+ replicated)
  int world, rank;
  long long cap;             // slots per block
  int rep_cap;               // slots for the replicated group
  const int32_t* err;        // the batch's validation word
  int32_t* ids;              // [(2W - 1) cap] local row per slot, -1 = empty
  int32_t* hdr;              // [(2W - 1) 4]: count, flags, sender rank, step (dl_shard_stamp)
  int32_t* rep_ids;          // [rep_cap] replicated rows (may be NULL when rep_cap == 0)
  int32_t* upos;             // [n_max] slot of each unique row (may be NULL), -1 = overflow
  int32_t* inv;              // [n_refs] inverse map, remapped in place to slots (may be NULL)
  long long n_refs, n_max;
};

// The slot of unique row u: owner group p (counts in LDS), index j within it.
__device__ __forceinline__ int route_slot(const RouteArgs& a, const long long* off, const int* cnt, long long u) {
  int p = 0;
  while (p < a.world && u >= off[p] + cnt[p]) ++p;
  const long long j = u - off[p];
  if (p < a.world) return j < a.cap ? (int)(shard_block(p, a.world, a.rank) * a.cap + j) : -1;
  return j < a.rep_cap ? (int)((2LL * a.world - 1) * a.cap + j) : -1;
}

__global__ __launch_bounds__(256) void shard_route_kernel(RouteArgs a) {
  __shared__ long long off[33];
  __shared__ int cnt[33];
  __shared__ int flags_s;
  const int W = a.world;
  if (threadIdx.x <= W) cnt[threadIdx.x] = a.counts[threadIdx.x];
  __syncthreads();
  if (threadIdx.x == 0) {
    long long o = 0;
    int ovf = 0;
    for (int p = 0; p <= W; ++p) {
      off[p] = o;
      o += cnt[p];
      ovf |= p < W ? cnt[p] > a.cap : cnt[p] > a.rep_cap;
    }
    flags_s = (a.err && a.err[0] ? DL_STATUS_BAD_ID : 0) | (ovf ? DL_STATUS_OVERFLOW : 0);
  }
  __syncthreads();
  const uint32_t mask = (1u << 27) - 1;
  if (blockIdx.x == 0 && threadIdx.x < W) {
    const int p = threadIdx.x;
    int32_t* h = a.hdr + shard_block(p, W, a.rank) * 4;
    h[0] = (int)min((long long)cnt[p], a.cap);
    h[1] = flags_s;
    h[2] = a.rank;
    h[3] = 0;
  }
  const long long nslots = W * a.cap + a.rep_cap;
  const long long nu = min((long long)a.n_uniq[0], a.n_max);
  const long long total = nslots + (a.upos ? a.n_max : 0) + (a.inv ? a.n_refs : 0);
  for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (long long)gridDim.x * blockDim.x) {
    if (t < W * a.cap) {                       // a request slot: the owner's j-th row, or empty
      const int p = (int)(t / a.cap);
      const long long j = t - p * a.cap;
      a.ids[shard_block(p, W, a.rank) * a.cap + j] = j < cnt[p] ? (int32_t)(a.uniq[off[p] + j] & mask) : -1;
    } else if (t < nslots) {                   // a replicated-row slot
      const long long j = t - W * a.cap;
      a.rep_ids[j] = j < cnt[W] ? (int32_t)(a.uniq[off[W] + j] & mask) : -1;
    } else if (a.upos && t < nslots + a.n_max) {
      const long long u = t - nslots;
      if (u < nu) a.upos[u] = route_slot(a, off, cnt, u);
    } else {                                   // the inverse map, in place
      const long long r = t - nslots - (a.upos ? a.n_max : 0);
      const int u = a.inv[r];
      if (u >= 0) a.inv[r] = route_slot(a, off, cnt, u);
    }
  }
}

// Just before the step's request exchange: every outgoing header gets this rank's sticky fault
// bits and the global step the step begins from (dl_shard_step_begin checks every rank agrees).
__global__ void shard_stamp_kernel(int32_t* __restrict__ hdr, int world, int rank, const float* __restrict__ opt) {
  const int p = threadIdx.x;
  if (p >= world) return;
  const int st = *opt_status(opt) & kStickyFaults;
  int32_t* h = hdr + shard_block(p, world, rank) * 4;
  h[1] |= st;
  h[3] = (int)opt[7];
}

static int grid_of(long long n) {
  long long g = (n + 255) / 256;
  if (g > 8192) g = 8192;
  return g < 1 ? 1 : (int)g;
}

}  // namespace dl

using namespace dl;

extern "C" int dl_shard_gather(const float* table, const float* first, const int32_t* ids, int64_t n,
                               int32_t emb_dim, float* out, float* out_first, void* stream) {
  DL_CHECK_ARG(table && ids && out && emb_dim % 4 == 0, "bad args");
  DL_CHECK_ARG(!first || out_first, "out_first required");
  if (n <= 0) return 0;
  hipLaunchKernelGGL(shard_gather_kernel, dim3(grid_of(n * (emb_dim / 4))), dim3(256), 0, as_stream(stream),
                     (const float4*)table, first, ids, (long long)n, emb_dim / 4, (float4*)out, out_first);
  DL_RETURN_LAUNCH("dl_shard_gather");
}

extern "C" int dl_shard_route(const uint32_t* uniq_keys, const int32_t* n_uniq, const int32_t* owner_counts,
                              int32_t world, int32_t rank, int64_t cap, int32_t rep_cap, const int32_t* err,
                              int32_t* ids, int32_t* hdr, int32_t* rep_ids, int32_t* upos, int32_t* inv,
                              int64_t n_refs, int64_t n_max, void* stream) {
  DL_CHECK_ARG(uniq_keys && n_uniq && owner_counts && ids && hdr, "NULL argument");
  DL_CHECK_ARG(world >= 1 && world <= 31 && rank >= 0 && rank < world, "bad world/rank");
  DL_CHECK_ARG(cap >= 1 && (2LL * world - 1) * cap + rep_cap < (1LL << 31), "bad capacity");
  DL_CHECK_ARG(rep_cap >= 0 && (rep_cap == 0 || rep_ids), "rep_ids required with rep_cap > 0");
  DL_CHECK_ARG(!inv || n_refs >= 0, "bad n_refs");
  RouteArgs a{uniq_keys, n_uniq, owner_counts, world, rank, (long long)cap, rep_cap, err, ids, hdr, rep_ids,
              upos, inv, inv ? (long long)n_refs : 0, upos ? (long long)n_max : 0};
  const long long total = world * cap + rep_cap + a.n_max + a.n_refs;
  hipLaunchKernelGGL(shard_route_kernel, dim3(grid_of(total)), dim3(256), 0, as_stream(stream), a);
  DL_RETURN_LAUNCH("dl_shard_route");
}

extern "C" int dl_shard_stamp(int32_t* hdr, int32_t world, int32_t rank, const float* opt, void* stream) {
  DL_CHECK_ARG(hdr && opt && world >= 1 && world <= 31 && rank >= 0 && rank < world, "bad args");
  hipLaunchKernelGGL(shard_stamp_kernel, dim3(1), dim3(64), 0, as_stream(stream), hdr, world, rank, opt);
  DL_RETURN_LAUNCH("dl_shard_stamp");
}

extern "C" int dl_shard_scatter_add(const float* g, const float* g_first, const int32_t* ids, int64_t n,
                                    int32_t emb_dim, float* G, float* G_first, uint8_t* touched, void* stream) {
  DL_CHECK_ARG(g && ids && G && touched, "bad args");
  if (n <= 0) return 0;
  hipLaunchKernelGGL(shard_scatter_kernel, dim3(grid_of(n * emb_dim)), dim3(256), 0, as_stream(stream), g, g_first,
                     ids, (long long)n, emb_dim, G, G_first, touched);
  DL_RETURN_LAUNCH("dl_shard_scatter_add");
}

extern "C" int dl_slab_sum(const float* slab, int32_t nslab, int64_t stride, int64_t n, float* out, void* stream) {
  DL_CHECK_ARG(slab && out && nslab >= 1 && stride >= n, "bad args");
  if (n <= 0) return 0;
  if (nslab >= 32 && n < 16384)
    hipLaunchKernelGGL(slab_sum_wave_kernel, dim3((unsigned)((n * 64 + 255) / 256)), dim3(256), 0, as_stream(stream),
                       slab, nslab, (long long)stride, (long long)n, out);
  else
    hipLaunchKernelGGL(slab_sum_kernel, dim3(grid_of(n)), dim3(256), 0, as_stream(stream), slab, nslab,
                       (long long)stride, (long long)n, out);
  DL_RETURN_LAUNCH("dl_slab_sum");
}

extern "C" int dl_keys_to_local(const uint32_t* keys, const int32_t* n_uniq, int64_t cap, int32_t* out,
                                void* stream) {
  DL_CHECK_ARG(keys && n_uniq && out, "bad args");
  if (cap <= 0) return 0;
  hipLaunchKernelGGL(keys_to_local_kernel, dim3(grid_of(cap)), dim3(256), 0, as_stream(stream), keys, n_uniq,
                     (long long)cap, out);
  DL_RETURN_LAUNCH("dl_keys_to_local");
}

extern "C" int dl_shard_gather_scalar(const float* w, const int32_t* ids, int64_t n, float* out, void* stream) {
  DL_CHECK_ARG(w && ids && out, "NULL argument");
  if (n <= 0) return 0;
  hipLaunchKernelGGL(shard_gather_scalar_kernel, dim3(grid_of(n)), dim3(256), 0, as_stream(stream), w, ids,
                     (long long)n, out);
  DL_RETURN_LAUNCH("dl_shard_gather_scalar");
}

extern "C" int dl_shard_add_fixed(const int64_t* g, const int32_t* ids, int64_t n, int64_t* G, uint8_t* touched,
                                  void* stream) {
  DL_CHECK_ARG(g && ids && G, "NULL argument");
  if (n <= 0) return 0;
  hipLaunchKernelGGL(shard_add_fixed_kernel, dim3(grid_of(n)), dim3(256), 0, as_stream(stream), g, ids, (long long)n,
                     G, touched);
  DL_RETURN_LAUNCH("dl_shard_add_fixed");
}

extern "C" int dl_wide_fold_owned(const float* gdeep, int32_t H, int64_t row0, int32_t world, int32_t rank, int64_t* G,
                                  uint8_t* touched, void* stream) {
  DL_CHECK_ARG(gdeep && G && H >= 0 && world >= 1 && rank >= 0 && rank < world, "bad args");
  if (H == 0) return 0;
  hipLaunchKernelGGL(wide_fold_owned_kernel, dim3(1), dim3(256), 0, as_stream(stream), gdeep, H, (long long)row0, world,
                     rank, G, touched);
  DL_RETURN_LAUNCH("dl_wide_fold_owned");
}

extern "C" int dl_wide_owned_values(const float* w, int32_t H, int64_t row0, int32_t world, int32_t rank, float* out,
                                    void* stream) {
  DL_CHECK_ARG(w && out && H >= 0 && world >= 1 && rank >= 0 && rank < world, "bad args");
  if (H == 0) return 0;
  hipLaunchKernelGGL(wide_owned_values_kernel, dim3(1), dim3(256), 0, as_stream(stream), w, H, (long long)row0, world,
                     rank, out);
  DL_RETURN_LAUNCH("dl_wide_owned_values");
}

extern "C" int dl_wide_local_ids(const int32_t* inv, int64_t n, int64_t offset, int64_t* out, void* stream) {
  DL_CHECK_ARG(inv && out, "NULL argument");
  if (n <= 0) return 0;
  hipLaunchKernelGGL(wide_local_ids_kernel, dim3(grid_of(n)), dim3(256), 0, as_stream(stream), inv, (long long)n,
                     (long long)offset, out);
  DL_RETURN_LAUNCH("dl_wide_local_ids");
}
