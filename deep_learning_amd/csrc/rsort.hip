// Stable LSD radix sort of (key, value) pairs for the batch index (rsort.h).
//
// Replaces hipcub::DeviceRadixSort (onesweep) in the index build.  Per pass over a digit of
// up to 9 bits (a 25-bit row key takes three passes: 9 + 8 + 8):
//   rs_upsweep    one block per 4096-element tile: digit histogram in LDS -> counts[d][tile]
//   rs_rowscan    one block per digit: exclusive scan of counts[d][*] in place, total[d]
//   rs_downsweep  one block per tile: every element's stable rank among the tile's elements
//                 of its digit (per-wave ballot match + per-wave LDS counters, waves in
//                 element order), the tile staged in LDS in digit order, then written out in
//                 runs: position = start of the digit + the tile's offset in it + index
// The first pass reads its pairs straight from the source (the batch's references: keys are
// computed from the ids, references without a key are dropped there), so the later passes
// and the unique step only ever see valid keys; their count stays on the device.
#include "rsort.h"

namespace dl {

constexpr int kRsThreads = 256;
constexpr int kRsWaves = kRsThreads / 64;
#ifndef DL_RS_ROUNDS
#define DL_RS_ROUNDS 16
#endif
// Elements per lane (a tile = 256 R elements).  Sorts of at least kRsBigN references use
// R = 12 with the keys materialised first (rs_keys_kernel): the downsweep then takes 36.9 KB of
// LDS and 68 VGPRs, so its blocks fit beside a forward s3 GEMM block on a CU (120 KB LDS,
// 2 x 200 VGPRs a SIMD) instead of holding CUs the GEMM's second round waits for
// (C3 4.43 -> 4.31 ms, C5 1.447 -> 1.437 ms; C2's 3.4 M candidate references: unchanged within
// the box's noise; profiles/r04z/, profiles/r04za/).
constexpr int kRsRounds = DL_RS_ROUNDS;
constexpr int kRsRoundsBig = 12;
#ifndef DL_RS_BIGN
#define DL_RS_BIGN (2LL << 20)
#endif
constexpr int64_t kRsBigN = DL_RS_BIGN;
#ifndef DL_RS_MAXBITS
#define DL_RS_MAXBITS 9
#endif
constexpr int kRsMaxBits = DL_RS_MAXBITS;                    // digit bits per pass at most
constexpr int kRsMaxRadix = 1 << kRsMaxBits;
constexpr int kLocal = 27;
constexpr uint32_t kRsNoKey = 0xFFFFFFFFu;   // rs_keys_kernel: a reference without a key
#ifndef DL_RS_PREKEYS
#define DL_RS_PREKEYS 0   // 1: keys materialised first by rs_keys_kernel at every size (always done from kRsBigN
#endif                    // on; below it, C2: alone 257 -> 246 us, in the step 7-20 us slower: profiles/r03pk/)

struct RsPass {
  int shift, bits;
  uint32_t lrange;
  const uint32_t* kin;        // passes after the first: input arrays
  const int32_t* vin;
  const int32_t* n_dev;       // valid count (after the first pass)
  int64_t n_max;
  int first;
};

__device__ __forceinline__ uint32_t rs_compress(uint32_t key, uint32_t lrange) {
  return lrange ? (key >> kLocal) * lrange + (key & ((1u << kLocal) - 1)) : key;
}

__device__ __forceinline__ int rs_digit(uint32_t key, const RsPass& p) {
  return (int)((rs_compress(key, p.lrange) >> p.shift) & ((1u << p.bits) - 1));
}

// The pair at element e of the pass's input; false when e has no key (or lies past the end).
// MODE 0: the previous pass's arrays; 1: the source's key array; 2: the batch's references;
// 3: the batch references' keys from rs_keys_kernel (value = the reference).
// Loads are unconditional (clamped index) and validity is computed after, so a tile's loads
// can all be in flight at once.
template <int MODE>
__device__ __forceinline__ bool rs_get(const RsSource& src, const RsPass& p, long long e, long long n, bool flag_err,
                                       uint32_t& key, int32_t& val) {
  const bool in = e < n;
  const long long ec = in ? e : 0;
  if (MODE == 0) {
    key = p.kin[ec];
    val = p.vin[ec];
    return in;
  }
  val = (int32_t)e;
  if (MODE == 1) {   // a negative int32 key (0xFFFFFFFF: a padding slot) is dropped
    key = src.keys[ec];
    return in && key != kRsNoKey;
  }
  if (MODE == 3) {   // keys materialised by rs_keys_kernel (kRsNoKey: no key)
    key = p.kin[ec];
    return in && key != kRsNoKey;
  }
  // the pair build's second id set: its layout's fields selected one by one (a selected
  // reference to a whole kernel-argument struct would be copied to scratch)
  const bool second = src.n1 > 0 && ec >= src.n1;
  const dl_emb_layout& L1 = src.L;
  const dl_emb_layout& L2 = src.L2;
  const int64_t* __restrict__ cate = second ? src.cate2 : src.cate;
  const int S = second ? L2.cate_fields : L1.cate_fields;
  const int use_fm = second ? L2.use_fm : L1.use_fm;
  const int ns = second ? index_slots(L2) : index_slots(L1);
  const int mb = second ? index_multi_base(L2) : index_multi_base(L1);
  const int cate_ld = second ? L2.cate_ld : L1.cate_ld;
  const int64_t n_rows = second ? L2.n_rows : L1.n_rows;
  const bool zero_row0 = second ? L2.zero_row0 : L1.zero_row0;
  // 32-bit division (a reference index is an int32): the 64-bit one is a long subroutine,
  // and this runs per element in both the upsweep and the downsweep
  const uint32_t ecu = (uint32_t)(second ? ec - src.n1 : ec), b = ecu / (uint32_t)ns;
  const int s = (int)(ecu - b * (uint32_t)ns);
  const int col = (use_fm && s < S) ? s : s < mb ? (use_fm ? s - S : s) : S + (s - mb);
  const int64_t off = (use_fm && s < S) ? (second ? L2.fm_cate_offset : L1.fm_cate_offset)
                                        : (second ? L2.deep_cate_offset : L1.deep_cate_offset);
  const int64_t row = cate[(long long)b * cate_ld + col] + off;
  const bool range_ok = row >= 0 && row < n_rows;
  if (in && !range_ok && flag_err && src.err) atomicOr(src.err, 1);
  const int w = src.world;
  const uint32_t r32 = (uint32_t)row;
  const uint32_t qw = w == 1 ? r32 : r32 / (uint32_t)w;   // w is uniform: one rank divides by nothing
  key = second ? ((1u << kLocal) | r32)
               : row < src.rep_below ? (((uint32_t)w << kLocal) | r32) : (((r32 - qw * (uint32_t)w) << kLocal) | qw);
  return in && range_ok && !(row == 0 && zero_row0);
}

// The batch references' keys, one streaming pass (MODE 3's input): the first sort pass then
// reads 4 B per candidate instead of gathering its int64 id and deriving the key twice (in the
// upsweep and again in the downsweep).  A reference without a key gets kRsNoKey, its inverse
// entry -1, and an out-of-range id flags the batch, as MODE 2's upsweep did.
__global__ __launch_bounds__(kRsThreads) void rs_keys_kernel(RsSource src, long long n, uint32_t* __restrict__ keys) {
  const RsPass p{};
  for (long long e = (long long)blockIdx.x * kRsThreads + threadIdx.x; e < n; e += (long long)gridDim.x * kRsThreads) {
    uint32_t key;
    int32_t val;
    const bool ok = rs_get<2>(src, p, e, n, true, key, val);
    keys[e] = ok ? key : kRsNoKey;
    if (!ok && src.inv) src.inv[e] = -1;
  }
}

__device__ __forceinline__ long long rs_count(const RsPass& p) {
  return p.first ? p.n_max : (long long)min((long long)*p.n_dev, p.n_max);
}

template <int MODE, int R>
__global__ __launch_bounds__(kRsThreads) void rs_upsweep(RsSource src, RsPass p, int32_t* __restrict__ counts,
                                                         int tiles) {
  constexpr int kRsTile = kRsThreads * R;
  __shared__ int hist[kRsMaxRadix];
  const int radix = 1 << p.bits;
  for (int d = threadIdx.x; d < radix; d += kRsThreads) hist[d] = 0;
  __syncthreads();
  const long long n = rs_count(p);
  const long long t0 = (long long)blockIdx.x * kRsTile;
  // every load of the tile first (one memory round trip), then the histogram
  uint32_t key[R];
  bool ok[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const long long e = t0 + r * kRsThreads + threadIdx.x;   // coalesced: counting needs no order
    int32_t val;
    ok[r] = rs_get<MODE>(src, p, e, n, true, key[r], val);
    if (MODE == 2 && !ok[r] && e < n && src.inv) src.inv[e] = -1;
  }
#pragma unroll
  for (int r = 0; r < R; ++r)
    if (ok[r]) atomicAdd(&hist[rs_digit(key[r], p)], 1);
  __syncthreads();
  for (int d = threadIdx.x; d < radix; d += kRsThreads) counts[(long long)d * tiles + blockIdx.x] = hist[d];
}

// Block-wide exclusive scan of one int per thread; returns the exclusive prefix, *total = sum.
__device__ __forceinline__ int rs_block_scan(int x, int* wsum, int* total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int inc = x;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(inc, o, 64);
    if (lane >= o) inc += y;
  }
  __syncthreads();
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  int base = 0, all = 0;
#pragma unroll
  for (int i = 0; i < kRsWaves; ++i) {
    base += i < w ? wsum[i] : 0;
    all += wsum[i];
  }
  *total = all;
  return base + inc - x;
}

// counts[d][0 .. tiles) -> exclusive offsets within the digit; total[d] = the digit's count
__global__ __launch_bounds__(kRsThreads) void rs_rowscan(int32_t* __restrict__ counts, int tiles,
                                                         int32_t* __restrict__ total) {
  __shared__ int wsum[kRsWaves];
  int32_t* row = counts + (long long)blockIdx.x * tiles;
  const int per = (tiles + kRsThreads - 1) / kRsThreads;
  const int a = threadIdx.x * per, b = min(tiles, a + per);
  // a thread's run of counts read 16 at a time, all in flight together (a serial loop paid one
  // memory round trip per count: C3's 16.6 k tiles a digit, 82 us a pass, profiles/r05p/)
  int s = 0;
  for (int i0 = a; i0 < b; i0 += 16) {
    int v[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = i0 + j < b ? row[i0 + j] : 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) s += v[j];
  }
  int all;
  int run = rs_block_scan(s, wsum, &all);
  for (int i0 = a; i0 < b; i0 += 16) {
    int v[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = i0 + j < b ? row[i0 + j] : 0;
#pragma unroll
    for (int j = 0; j < 16; ++j)
      if (i0 + j < b) {
        row[i0 + j] = run;
        run += v[j];
      }
  }
  if (threadIdx.x == 0) total[blockIdx.x] = all;
}

template <int MODE, int R>
__global__ __launch_bounds__(kRsThreads) void rs_downsweep(RsSource src, RsPass p, const int32_t* __restrict__ counts,
                                                           int tiles, const int32_t* __restrict__ total,
                                                           uint32_t* __restrict__ kout, int32_t* __restrict__ vout,
                                                           int32_t* __restrict__ n_valid) {
  constexpr int kRsTile = kRsThreads * R, kRsWaveSpan = 64 * R;   // tile; consecutive elements per wave
  __shared__ int cnt[kRsWaves][kRsMaxRadix];   // per-wave running counts, then per-wave prefixes
  __shared__ int tstart[kRsMaxRadix];          // the tile's digit starts (exclusive scan over digits)
  __shared__ int gbase[kRsMaxRadix];           // global position of the tile's first element of each digit
  __shared__ uint32_t sk[kRsTile];
  __shared__ int32_t sv[kRsTile];
  __shared__ int wsum[kRsWaves];
  __shared__ int tile_n;
  const int radix = 1 << p.bits;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const long long n = rs_count(p);
  const long long e0 = (long long)blockIdx.x * kRsTile + (long long)w * kRsWaveSpan;
  uint32_t key[R];
  int32_t val[R];
  int rank[R];
  const uint64_t lt = (1ull << lane) - 1;
  // every load of the wave's 1024 elements first (one memory round trip)
  uint32_t okm = 0;
#pragma unroll
  for (int r = 0; r < R; ++r)
    okm |= rs_get<MODE>(src, p, e0 + r * 64 + lane, n, false, key[r], val[r]) ? (1u << r) : 0u;
  for (int i = tid; i < kRsWaves * kRsMaxRadix; i += kRsThreads) (&cnt[0][0])[i] = 0;
  // digit starts from the totals (each thread scans two digits' worth)
  {
    const int d0 = 2 * tid;
    const int a = d0 < radix ? total[d0] : 0, b = d0 + 1 < radix ? total[d0 + 1] : 0;
    int all;
    const int ex = rs_block_scan(a + b, wsum, &all);
    if (d0 < radix) gbase[d0] = ex;
    if (d0 + 1 < radix) gbase[d0 + 1] = ex + a;
    if (p.first && blockIdx.x == 0 && tid == 0 && n_valid) *n_valid = all;
  }
  __syncthreads();
  for (int d = tid; d < radix; d += kRsThreads) gbase[d] += counts[(long long)d * tiles + blockIdx.x];
  // per-wave stable ranks: rounds in element order, lanes in element order within a round
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const bool ok = (okm >> r) & 1;
    const int d = ok ? rs_digit(key[r], p) : 0;
    uint64_t peers = __ballot(ok);
    for (int b = 0; b < p.bits; ++b) {
      const bool bit = (d >> b) & 1;
      const uint64_t bb = __ballot(bit);
      peers &= bit ? bb : ~bb;
    }
    int base = 0;
    if (ok) base = cnt[w][d];
    rank[r] = ok ? base + __popcll(peers & lt) : -1;
    // the lowest lane of each digit group advances the wave's counter (LDS ops of one wave
    // execute in order: every lane's read above lands before this write)
    if (ok && (peers & lt) == 0) cnt[w][d] = base + __popcll(peers);
  }
  __syncthreads();
  // per-digit: wave prefixes (in place) and the tile's count, then the tile-local digit starts
  {
    int tc[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int d = 2 * tid + j;
      int run = 0;
      if (d < radix) {
#pragma unroll
        for (int ww = 0; ww < kRsWaves; ++ww) {
          const int c = cnt[ww][d];
          cnt[ww][d] = run;
          run += c;
        }
      }
      tc[j] = run;
    }
    int all;
    const int ex = rs_block_scan(tc[0] + tc[1], wsum, &all);
    if (2 * tid < radix) tstart[2 * tid] = ex;
    if (2 * tid + 1 < radix) tstart[2 * tid + 1] = ex + tc[0];
    if (tid == 0) tile_n = all;
  }
  __syncthreads();
  // stage the tile in digit order
#pragma unroll
  for (int r = 0; r < R; ++r) {
    if (rank[r] >= 0) {
      const int d = rs_digit(key[r], p);
      const int lp = tstart[d] + cnt[w][d] + rank[r];
      sk[lp] = key[r];
      sv[lp] = val[r];
    }
  }
  __syncthreads();
  // write out in runs: consecutive threads -> consecutive positions within a digit
  const int tn = tile_n;
  for (int i = tid; i < tn; i += kRsThreads) {
    const uint32_t k = sk[i];
    const int d = rs_digit(k, p);
    const long long pos = (long long)gbase[d] + (i - tstart[d]);
    kout[pos] = k;
    vout[pos] = sv[i];
  }
}

static size_t rs_align(size_t x) { return (x + 255) & ~(size_t)255; }

static int rs_rounds(int64_t n) { return n >= kRsBigN ? kRsRoundsBig : kRsRounds; }
static int rs_tiles(int64_t n) { return (int)((n + kRsThreads * rs_rounds(n) - 1) / (kRsThreads * rs_rounds(n))); }

size_t rsort_workspace_bytes(int64_t n) {
  if (n < 1) n = 1;
  const int tiles = rs_tiles(n);
  return 2 * rs_align((size_t)n * 4) + rs_align((size_t)kRsMaxRadix * tiles * 4) + rs_align(kRsMaxRadix * 4);
}

// one pass: tile histograms, their scan per digit, the stable scatter
template <int R>
static void rs_pass(int mode, const RsSource& src, const RsPass& p, int32_t* counts, int tiles, int32_t* total, int pb,
                    uint32_t* ko, int32_t* vo, int32_t* n_valid, hipStream_t s) {
  if (mode == 0) hipLaunchKernelGGL((rs_upsweep<0, R>), dim3(tiles), dim3(kRsThreads), 0, s, src, p, counts, tiles);
  else if (mode == 1) hipLaunchKernelGGL((rs_upsweep<1, R>), dim3(tiles), dim3(kRsThreads), 0, s, src, p, counts, tiles);
  else if (mode == 2) hipLaunchKernelGGL((rs_upsweep<2, R>), dim3(tiles), dim3(kRsThreads), 0, s, src, p, counts, tiles);
  else hipLaunchKernelGGL((rs_upsweep<3, R>), dim3(tiles), dim3(kRsThreads), 0, s, src, p, counts, tiles);
  hipLaunchKernelGGL(rs_rowscan, dim3(1 << pb), dim3(kRsThreads), 0, s, counts, tiles, total);
  if (mode == 0)
    hipLaunchKernelGGL((rs_downsweep<0, R>), dim3(tiles), dim3(kRsThreads), 0, s, src, p, counts, tiles, total, ko, vo, n_valid);
  else if (mode == 1)
    hipLaunchKernelGGL((rs_downsweep<1, R>), dim3(tiles), dim3(kRsThreads), 0, s, src, p, counts, tiles, total, ko, vo, n_valid);
  else if (mode == 2)
    hipLaunchKernelGGL((rs_downsweep<2, R>), dim3(tiles), dim3(kRsThreads), 0, s, src, p, counts, tiles, total, ko, vo, n_valid);
  else
    hipLaunchKernelGGL((rs_downsweep<3, R>), dim3(tiles), dim3(kRsThreads), 0, s, src, p, counts, tiles, total, ko, vo, n_valid);
}

int rsort_pairs(const RsSource& src, int64_t n, uint32_t lrange, int bits, void* ws, size_t ws_bytes,
                uint32_t* out_keys, int32_t* out_vals, int32_t* n_valid, hipStream_t s) {
  if (n <= 0) return 0;
  if (ws_bytes < rsort_workspace_bytes(n) || bits < 1 || bits > 32 || !n_valid) return 22;
  const int tiles = rs_tiles(n);
  char* w = reinterpret_cast<char*>(ws);
  uint32_t* tk = reinterpret_cast<uint32_t*>(w); w += rs_align((size_t)n * 4);
  int32_t* tv = reinterpret_cast<int32_t*>(w); w += rs_align((size_t)n * 4);
  int32_t* counts = reinterpret_cast<int32_t*>(w); w += rs_align((size_t)kRsMaxRadix * tiles * 4);
  int32_t* total = reinterpret_cast<int32_t*>(w);
  // digit width: up to 9 bits a pass; for large sorts (C3's 51 M candidate references) at
  // most 8 — one more pass, but longer runs per digit in each tile's scatter (25-bit keys:
  // 7/6/6/6 instead of 9/8/8; C3 index 1,033 -> 871 us, step 4.48 -> 4.39 ms), while C2's
  // 3.4 M-pair sort measured slower as a step with the extra pass (profiles/r03t/)
  const int maxb = n >= (int64_t)(8 << 20) ? min(8, kRsMaxBits) : kRsMaxBits;
  const int passes = (bits + maxb - 1) / maxb;
  int shift = 0;
  const uint32_t* kin = nullptr;
  const int32_t* vin = nullptr;
  for (int i = 0; i < passes; ++i) {
    const int pb = (bits - shift + (passes - i) - 1) / (passes - i);   // spread the bits evenly
    // the last pass lands in the outputs: alternate backwards from it
    const bool to_out = ((passes - 1 - i) & 1) == 0;
    uint32_t* ko = to_out ? out_keys : tk;
    int32_t* vo = to_out ? out_vals : tv;
    RsPass p{shift, pb, lrange, kin, vin, n_valid, n, i == 0 ? 1 : 0};
    int mode = i > 0 ? 0 : src.kind == 0 ? 1 : 2;
    if (mode == 2 && (DL_RS_PREKEYS || n >= kRsBigN)) {
      // the keys into a buffer pass 0 does not write: out_keys when pass 0 lands in the
      // temporaries, else the temporary keys (the first pass's output is the outputs)
      uint32_t* pre = to_out ? tk : out_keys;
      long long g = ((long long)n + kRsThreads - 1) / kRsThreads;
      if (g > 8192) g = 8192;
      hipLaunchKernelGGL(rs_keys_kernel, dim3((unsigned)g), dim3(kRsThreads), 0, s, src, (long long)n, pre);
      p.kin = pre;
      mode = 3;
    }
    if (rs_rounds(n) == kRsRoundsBig)
      rs_pass<kRsRoundsBig>(mode, src, p, counts, tiles, total, pb, ko, vo, n_valid, s);
    else
      rs_pass<kRsRounds>(mode, src, p, counts, tiles, total, pb, ko, vo, n_valid, s);
    kin = ko;
    vin = vo;
    shift += pb;
  }
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

}  // namespace dl
