// Embedding gather / FM / multi-hot pooling kernels (forward and backward).
//
// Reference semantics (paths relative to the reference repo):
//   models/deepfm_pipeline.py:83-123   row-0 zero, dual FM/deep indexing, FM 1st/2nd order
//   models/deepfm_multi_cate.py:71-111 nonzero-mean pooling of multi-hot slots
//   models/dnn_pipeline.py:72-83, models/wdl.py:132-179 deep lookups
//
// Layout on the MI355X:
//   forward  — one wave per sample; a table row of E floats is read by E/4 lanes
//              as float4 (E=16: 64 B row = 4 lanes, 16 rows per wave
//              instruction); the FM sums reduce over the row lanes with
//              xor-shuffles, nothing is materialised in HBM except the outputs.
//   backward — one wave per sample; a row is E lanes x 4 B so every atomic
//              wave instruction adds whole rows (E=16: 4 rows x 64 B); the hot
//              cont-field rows (hit by every sample) accumulate in registers
//              and leave the block once as a partial slab.
#include "common.h"
#include "rec.h"
#include "segment.h"

namespace dl {

struct EmbArgs {
  dl_emb_layout L;
  const int32_t* inv;      // indexed mode (sharded): row of a reference = inv_base + inv[ref]
  int inv_base;
  const float* table;
  const float* first_order;
  const int64_t* cate;
  const float* cont;
  const float* vec;
  float* x0;
  float* fm_out;
  float* fm_sum;
  int32_t* err;
  // record mode (single GPU, lazy Adam): the cate rows are read straight from the row
  // records and caught up to step opt[7] - lag in registers; `table` / `first_order`
  // then hold only the C replicated FM cont-field rows (compact, caught up by dl_rec_gather)
  const float* rec;
  RecCfg rc;
  const float* hist;
  const float* opt;
  int lag;
  // staged mode (with inv; the lazy single-GPU forward after dl_rec_gather_scatter): the FM
  // reference (b, f) reads table row inv_base + b*S + f (the FM staging rows), its first-order
  // output and the deep references' x0 columns are already written — only references whose
  // row has no key (inv < 0: the zero row) are written here, as zeros
  int staged;
  // (dl_embed_fwd_gtab) the deep references' row byte offsets for the fused first tower layer,
  // common.h kGtab* layout; the deep rows themselves are then not read here
  uint32_t* gtab;
};

__device__ __forceinline__ bool row_ok(int64_t row, int zero_row0) {
  return row > 0 || (row == 0 && !zero_row0);
}

__device__ __forceinline__ float4 f4_zero() { return make_float4(0.f, 0.f, 0.f, 0.f); }

constexpr int kMaxHotContFwd = 32;

constexpr int kTileSamples = 16;   // samples staged per block iteration
constexpr int kGtabMaxNps = 4;     // dl_embed_fwd_gtab: at most 4 passes of FM slots a sample
constexpr int kMaxSlots = 128;     // FM slots + deep slots per sample

#ifndef DL_FWD_SPW
#define DL_FWD_SPW 1   // samples a wave keeps in flight in the plain / slot lookups (see the kernel)
#endif
#ifndef DL_FWD_MIN_WAVES
#define DL_FWD_MIN_WAVES 5
#endif
// Occupancy: NPS <= 4 fits 5 waves a SIMD (83-92 VGPRs); the NPS = 5 forms (C2's full lookup: 13 +
// 26 FM + 26 deep slots) need 100 VGPRs — at 5 waves they spilled 3, so they take 4 (the plain
// slot-plane lookup 131.7 -> 128.5 us uniform, 92.5 -> 90.8 Zipf, profiles/r06z5/); NPS > 5: unbounded.
#ifndef DL_POOL_DIAG_NO_W1
#define DL_POOL_DIAG_NO_W1 0   // diagnostics build: first-order weights not read by the forward / pooling (wrong fm_out)
#endif
#ifndef DL_POOL_DIAG
#define DL_POOL_DIAG 0   // diagnostics builds (wrong results; the compacted pooling): 1 = every row read from row 0
#endif                   // (cache-resident), 2 = no pooled / count / first-order output stores
// REC: 0 dense table; 1 row records caught up in registers (lazy training); 2 row records
// already caught up (a flushed table: predict after dl_rec_flush) — only each record's first
// 128-B line is read (p and the first-order triple + stamp), a stale row faults (DL_STATUS_LAG).
template <int E, int NPS, int REC = 0>
// (two samples in flight a wave, DL_FWD_SPW below: 4 waves a SIMD, up to 128 VGPRs)
__global__ __launch_bounds__(256, (REC == 1 || NPS > 5) ? 1
                                  : (NPS == 5 || (DL_FWD_SPW > 1 && (REC == 0 || REC == 3) && NPS <= 3)) ? 4
                                  : DL_FWD_MIN_WAVES)
void embed_fwd_kernel(EmbArgs a) {
  // Per block iteration a tile of 16 samples is staged: every (sample, slot)
  // row index is resolved once into LDS by a coalesced pass over the id matrix
  // (slot = FM field f < Fs, or deep field Fs + f).  Each wave then owns 4
  // samples; for a sample it issues ALL its row loads back to back (packed
  // slots, E/4 lanes per row, float4 per lane) before consuming any, so a wave
  // keeps a whole sample's rows in flight.  Masked slots read row 0 and are
  // zeroed by select, never by a branch around the load.
  constexpr int LPR = E / 4;
  constexpr int RPI = 64 / LPR;
  constexpr bool RECS = REC == 1 || REC == 2;          // the record modes
  constexpr int TP = REC == 3 ? 2 * LPR : LPR;         // float4s between table rows (slot plane: 2E floats)
  constexpr int W1S = REC == 3 ? 2 * E : 1;            // floats between first-order weights
  __shared__ int rows_s[kTileSamples][kMaxSlots];
  __shared__ float vals_s[kTileSamples][kMaxHotContFwd];
  const dl_emb_layout& L = a.L;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int r = lane / LPR, q = lane % LPR;
  const int Cf = (L.use_fm && L.fm_cont) ? L.cont_fields : 0;
  const int S = L.cate_fields;
  const int Fs = L.use_fm ? Cf + S : 0;
  const int F = Fs + L.fm_extra;
  const int nslot = Fs + (L.x0_cat_col >= 0 ? S : 0);   // -1: the deep rows are not looked up here
  const float4* tab4 = reinterpret_cast<const float4*>(a.table);
  const float4 z4 = f4_zero();
  const int ntiles = (L.batch + kTileSamples - 1) / kTileSamples;
  RecCfg rc = a.rc;
  int target = 0;
  extern __shared__ float hist_s[];   // record mode: the alpha ring, so the catch-up loop's
                                      // per-step reads are LDS hits, not L2 round trips
  if (REC == 2) {
    target = (int)a.opt[7] - a.lag;
    rc.status = opt_status(a.opt);
  }
  if (REC == 1) {
    rec_load_hyper(rc, a.opt);
    target = (int)a.opt[7] - a.lag;
    for (int k = threadIdx.x; k <= rc.hist_mask; k += blockDim.x) hist_s[k] = a.hist[k];
    __syncthreads();
  }

  for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int b0 = t * kTileSamples;
    const int nb = min(kTileSamples, L.batch - b0);
    // stage row indices: one id feeds its FM slot (Cf + f) and its deep slot (Fs + f).
    // Loads are unconditional (clamped index) so all of a thread's id loads are in flight together.
    {
      const int tot = nb * S;
      if (a.inv) {
        // sharded: rows were exchanged per unique reference; ref = b * ns + slot
        const int ns = index_slots(L);
        for (int k = threadIdx.x; k < tot; k += blockDim.x) {
          const int j = k / S, f = k % S;
          const int64_t rb = (int64_t)(b0 + j) * ns;
          const int di = a.inv[rb + (L.use_fm ? S : 0) + f];
          rows_s[j][Fs + f] = di < 0 ? -1 : (a.staged ? -2 : a.inv_base + di);   // -2: written by the gather
          if (L.use_fm) {
            const int fi = a.inv[rb + f];
            rows_s[j][Cf + f] = fi < 0 ? -1 : a.inv_base + (a.staged ? (b0 + j) * S + f : fi);
          }
        }
      } else {
        for (int k0 = 0; k0 < tot; k0 += 4 * 256) {
          int64_t idv[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            int k = k0 + threadIdx.x + u * 256;
            k = k < tot ? k : tot - 1;
            idv[u] = a.cate[(int64_t)(b0 + k / S) * L.cate_ld + k % S];
          }
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int k = k0 + threadIdx.x + u * 256;
            if (k < tot) {
              const int j = k / S, f = k % S;
              const int dr = (int)checked_row(idv[u], L.deep_cate_offset, L.n_rows, a.err);
              rows_s[j][Fs + f] = row_ok(dr, L.zero_row0) ? dr : -1;
              if (L.use_fm) {
                const int fr = (int)checked_row(idv[u], L.fm_cate_offset, L.n_rows, a.err);
                rows_s[j][Cf + f] = row_ok(fr, L.zero_row0) ? fr : -1;
              }
            }
          }
        }
      }
      for (int k = threadIdx.x; k < nb * Cf; k += blockDim.x) {
        const int64_t row = L.fm_cont_offset + k % Cf;   // compact: rows 0..C-1 of the gathered rows
        rows_s[k / Cf][k % Cf] = row_ok(row, L.zero_row0) ? (L.cont_rows_compact ? k % Cf : (int)row) : -1;
      }
    }
    for (int k = threadIdx.x; k < nb * Cf; k += blockDim.x)
      vals_s[k / Cf][k % Cf] = a.cont[(int64_t)(b0 + k / Cf) * L.cont_fields + k % Cf];
    __syncthreads();
    // (the instantiations the gtab lookup launches: with x0_cat_col = -1 a sample's slots are its
    // FM fields only; instantiated in the others it costs the NPS = 5 forms spilled registers)
    if constexpr ((REC == 0 || REC == 3) && NPS <= kGtabMaxNps) if (a.gtab) {
      // the tile's deep rows as byte offsets, field-major: 16 samples = one 64-B piece a field
      // (a tile never straddles two 256-sample tables: kGtabRows % kTileSamples == 0)
      uint32_t* gt = a.gtab + (int64_t)(b0 / kGtabRows) * S * kGtabPitch + b0 % kGtabRows;
      const uint32_t rb = 16u * (uint32_t)TP;   // bytes between plane rows
      for (int k = threadIdx.x; k < S * kTileSamples; k += blockDim.x) {
        const int f = k / kTileSamples, j = k % kTileSamples;
        if (j < nb) {
          const int dr = rows_s[j][Fs + f];
          gt[f * kGtabPitch + j] = dr >= 0 ? (uint32_t)dr * rb : kGtabMasked;
        }
      }
    }
    // SPW samples per wave iteration, all their row loads issued before any is consumed
    // (DL_FWD_SPW = 2: the plain / slot-plane lookups with at most 3 passes a sample; measured
    // neutral on the FM-only lookup of the fused predict, 60 us both, profiles/r06i): one
    constexpr int SPW = DL_FWD_SPW > 1 && (REC == 0 || REC == 3) && NPS <= 3 ? DL_FWD_SPW : 1;
    for (int jw = wid; jw < nb; jw += 4 * SPW) {
      float4 v[SPW][NPS];
      int rw[SPW][NPS];
      float w1[SPW], val[SPW];
      int frow[SPW];
      bool w1_done[SPW];
#pragma unroll
      for (int u = 0; u < SPW; ++u) {
        const int j = min(jw + 4 * u, nb - 1);   // past the tile: repeats its last sample, not written
        const int b = b0 + j;
#pragma unroll
        for (int p = 0; p < NPS; ++p) {
          const int sl = p * RPI + r;
          rw[u][p] = rows_s[j][sl < nslot ? sl : 0];
          if (sl >= nslot) rw[u][p] = -1;
        }
        if (!RECS) {
#pragma unroll
          for (int p = 0; p < NPS; ++p) v[u][p] = tab4[(int64_t)(rw[u][p] < 0 ? 0 : rw[u][p]) * TP + q];
        } else if (REC == 2) {
          float4 t4[NPS];
#pragma unroll
          for (int p = 0; p < NPS; ++p) {
            const int sl = p * RPI + r;
            if (sl < Cf) {
              v[u][p] = tab4[(rw[u][p] < 0 ? 0 : rw[u][p]) * LPR + q];
            } else {
              const float* rr = a.rec + (int64_t)(rw[u][p] < 0 ? 0 : rw[u][p]) * rc.ld;
              v[u][p] = *reinterpret_cast<const float4*>(rr + 4 * q);
              t4[p] = *reinterpret_cast<const float4*>(rr + E);
            }
          }
#pragma unroll
          for (int p = 0; p < NPS; ++p) {
            const int sl = p * RPI + r;
            if (sl >= Cf && sl < nslot) {
              if (rw[u][p] >= 0 && __float_as_int(t4[p].w) != target) raise_fault(rc.status, DL_STATUS_LAG);
              if (sl < Fs && rc.has_first && q == 0) a.fm_out[(int64_t)b * L.fm_ld + sl] = rw[u][p] < 0 ? 0.f : t4[p].x * 1.f;
            }
          }
        } else {
          // slots >= Cf: the whole record (p, m, v, first-order triple + stamp) is loaded for
          // every pass before any is consumed, then caught up exactly as dl_rec_gather does
          // (same catch_up4 on the same float4): the values are bit-identical to the
          // gathered rows the indexed forward reads.
          float4 m4[NPS], v4[NPS], t4[NPS];
#pragma unroll
          for (int p = 0; p < NPS; ++p) {
            const int sl = p * RPI + r;
            if (sl < Cf) {
              v[u][p] = tab4[(rw[u][p] < 0 ? 0 : rw[u][p]) * LPR + q];
            } else {
              const float* rr = a.rec + (int64_t)(rw[u][p] < 0 ? 0 : rw[u][p]) * rc.ld;
              v[u][p] = *reinterpret_cast<const float4*>(rr + 4 * q);
              m4[p] = *reinterpret_cast<const float4*>(rr + E + 4 + 4 * q);
              v4[p] = *reinterpret_cast<const float4*>(rr + 2 * E + 4 + 4 * q);
              t4[p] = *reinterpret_cast<const float4*>(rr + E);
            }
          }
#pragma unroll
          for (int p = 0; p < NPS; ++p) {
            const int sl = p * RPI + r;
            if (sl >= Cf && sl < nslot) {
              const bool fmf = sl < Fs && rc.has_first && q == 0;   // FM slot: its first-order weight too
              float w = t4[p].x, wm = t4[p].y, wv = t4[p].z;
              const int stamp = __float_as_int(t4[p].w);
              if (stamp < target) catch_up4(v[u][p], m4[p], v4[p], w, wm, wv, fmf, stamp, target, RingG{hist_s, rc.hist_mask}, rc);
              if (fmf) a.fm_out[(int64_t)b * L.fm_ld + sl] = rw[u][p] < 0 ? 0.f : w * 1.f;
            }
          }
        }
        // first-order terms (one lane per FM field; record mode: the cont fields only)
        w1[u] = 0.f;
        val[u] = 0.f;
        frow[u] = -1;
        // staged: the FM cate fields' first-order outputs were written by the gather (their rows
        // index the staging rows, not first_order) — only the zero rows' are written here
        w1_done[u] = a.staged && lane >= Cf && lane < Fs && rows_s[j][lane] >= 0;
        if (lane < (RECS ? Cf : Fs)) {
          frow[u] = rows_s[j][lane];
          val[u] = lane < Cf ? vals_s[j][lane] : 1.f;
          w1[u] = DL_POOL_DIAG_NO_W1 ? 1.f : a.first_order[(int64_t)((frow[u] < 0 || w1_done[u]) ? 0 : frow[u]) * W1S];
        }
      }
#pragma unroll
      for (int u = 0; u < SPW; ++u) {
      const int j = jw + 4 * u;
      if (u > 0 && j >= nb) break;   // wave-uniform
      const int b = b0 + j;
      float* xb = a.x0 + (int64_t)b * L.x0_ld;
      // bf16 x0 (L.x0_bf16): the same columns, as bf16 (a.x0 then points at uint16 storage)
      unsigned short* xbb = reinterpret_cast<unsigned short*>(a.x0) + (int64_t)b * L.x0_ld;
      float4 s = z4, ss = z4;
#pragma unroll
      for (int p = 0; p < NPS; ++p) {
        {
          const int sl = p * RPI + r;
          const float4 t4 = rw[u][p] < 0 ? z4 : v[u][p];
          if (sl < Fs) {
            const float vv = sl < Cf ? vals_s[j][sl] : 1.f;
            // explicit roundings (no contraction left to the compiler): every instantiation
            // of this kernel (table, indexed, record) must produce the same FM sums
            const float4 ev = make_float4(__fmul_rn(t4.x, vv), __fmul_rn(t4.y, vv), __fmul_rn(t4.z, vv),
                                          __fmul_rn(t4.w, vv));
            s.x += ev.x; s.y += ev.y; s.z += ev.z; s.w += ev.w;
            ss.x = fmaf(ev.x, ev.x, ss.x); ss.y = fmaf(ev.y, ev.y, ss.y);
            ss.z = fmaf(ev.z, ev.z, ss.z); ss.w = fmaf(ev.w, ev.w, ss.w);
          } else if (sl < nslot && rw[u][p] != -2) {
            const int col = L.x0_cat_col + (sl - Fs) * E + 4 * q;
            if (L.x0_bf16)
              *reinterpret_cast<uint2*>(xbb + col) = make_uint2(f2bf(t4.x) | ((unsigned)f2bf(t4.y) << 16),
                                                                f2bf(t4.z) | ((unsigned)f2bf(t4.w) << 16));
            else
              *reinterpret_cast<float4*>(xb + col) = t4;
          }
        }
      }
      if (lane < (RECS ? Cf : Fs) && !w1_done[u]) a.fm_out[(int64_t)b * L.fm_ld + lane] = frow[u] < 0 ? 0.f : w1[u] * val[u];
      for (int f = 64 + lane; f < (RECS ? 0 : Fs); f += 64) {   // > 64 FM fields (rare; record mode: <= 64)
        const int fr = rows_s[j][f];
        if (a.staged && f >= Cf && fr >= 0) continue;
        const float vv = f < Cf ? vals_s[j][f] : 1.f;
        a.fm_out[(int64_t)b * L.fm_ld + f] = fr < 0 ? 0.f : a.first_order[(int64_t)fr * W1S] * vv;
      }
      if (L.use_fm) {
        for (int f0 = 0; f0 < L.fm_extra; f0 += RPI) {
          const int f = f0 + r;
          if (f < L.fm_extra) {
            const float4 ev = *reinterpret_cast<const float4*>(xb + L.x0_pool_col + f * E + 4 * q);
            s.x += ev.x; s.y += ev.y; s.z += ev.z; s.w += ev.w;
            ss.x = fmaf(ev.x, ev.x, ss.x); ss.y = fmaf(ev.y, ev.y, ss.y);
            ss.z = fmaf(ev.z, ev.z, ss.z); ss.w = fmaf(ev.w, ev.w, ss.w);
          }
        }
#pragma unroll
        for (int o = LPR; o < 64; o <<= 1) {
          s.x += __shfl_xor(s.x, o, 64); s.y += __shfl_xor(s.y, o, 64);
          s.z += __shfl_xor(s.z, o, 64); s.w += __shfl_xor(s.w, o, 64);
          ss.x += __shfl_xor(ss.x, o, 64); ss.y += __shfl_xor(ss.y, o, 64);
          ss.z += __shfl_xor(ss.z, o, 64); ss.w += __shfl_xor(ss.w, o, 64);
        }
        if (r == 0) {
          float* fo = a.fm_out + (int64_t)b * L.fm_ld + F + 4 * q;
          fo[0] = 0.5f * fmaf(s.x, s.x, -ss.x); fo[1] = 0.5f * fmaf(s.y, s.y, -ss.y);
          fo[2] = 0.5f * fmaf(s.z, s.z, -ss.z); fo[3] = 0.5f * fmaf(s.w, s.w, -ss.w);
          if (a.fm_sum) *reinterpret_cast<float4*>(a.fm_sum + (int64_t)b * E + 4 * q) = s;
        }
      }
      if (L.x0_cont_col >= 0)
        for (int jj = lane; jj < L.cont_fields; jj += 64) {
          const float c = a.cont[(int64_t)b * L.cont_fields + jj];
          if (L.x0_bf16) xbb[L.x0_cont_col + jj] = f2bf(c); else xb[L.x0_cont_col + jj] = c;
        }
      if (L.x0_vec_col >= 0)
        for (int jj = lane; jj < L.vector_size; jj += 64) {
          const float c = a.vec[(int64_t)b * L.vector_size + jj];
          if (L.x0_bf16) xbb[L.x0_vec_col + jj] = f2bf(c); else xb[L.x0_vec_col + jj] = c;
        }
      }
    }
    __syncthreads();
  }
}

struct EmbBwdArgs {
  dl_emb_layout L;
  const float* table;
  const int64_t* cate;
  const float* cont;
  const float* dz;
  const float* w_head;
  const float* fm_sum;
  const float* dx0;
  float* g_table;
  float* g_first;
  uint8_t* touched;
  float* cont_slab;
};

constexpr int kMaxHotCont = 32;  // cont fields kept in registers on the backward

template <int E, bool CONT_ONLY>
__global__ __launch_bounds__(256) void embed_bwd_kernel(EmbBwdArgs a) {
  constexpr int RPI = 64 / E;  // rows per wave instruction (lane = dim)
  constexpr int NCP = (kMaxHotCont + RPI - 1) / RPI;
  const dl_emb_layout& L = a.L;
  const int lane = threadIdx.x & 63;
  const int r = lane / E, d = lane % E;
  const int wid = threadIdx.x >> 6;
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int nwaves = (gridDim.x * blockDim.x) >> 6;
  const int Cf = (L.use_fm && L.fm_cont) ? L.cont_fields : 0;
  const int S = L.cate_fields;
  const int Fs = Cf + S;
  const int F = Fs + L.fm_extra;

  float gc[NCP];
#pragma unroll
  for (int p = 0; p < NCP; ++p) gc[p] = 0.f;
  float g1c = 0.f;

  for (int b = wave; b < L.batch; b += nwaves) {
    const int64_t* ids = a.cate + (int64_t)b * L.cate_ld;
    if (L.use_fm) {
      const float dzb = a.dz[b];
      const float* cb = a.cont + (int64_t)b * L.cont_fields;
      const float dsec = dzb * a.w_head[F + d];
      const float sd = a.fm_sum[(int64_t)b * E + d];
      // hot cont-field rows: register accumulation
#pragma unroll
      for (int p = 0; p < NCP; ++p) {
        const int f = p * RPI + r;
        if (p * RPI < Cf && f < Cf) {
          const int64_t row = L.fm_cont_offset + f;
          const float val = cb[f];
          const float e = row_ok(row, L.zero_row0) ? a.table[(L.cont_rows_compact ? f : row) * E + d] * val : 0.f;
          gc[p] += val * dsec * (sd - e);
        }
      }
      // single cate FM fields: scatter-add
      for (int f0 = 0; f0 < (CONT_ONLY ? 0 : S); f0 += RPI) {
        const int f = f0 + r;
        if (f < S) {
          const int64_t row = ids[f] + L.fm_cate_offset;
          if (row < L.n_rows && row_ok(row, L.zero_row0)) {
            const float e = a.table[row * E + d];
            atomicAdd(a.g_table + row * E + d, dsec * (sd - e));
            if (d == 0) a.touched[row] = 1;
          }
        }
      }
      for (int f = lane; f < Fs; f += 64) {
        if (f < Cf) {
          g1c += dzb * a.w_head[f] * cb[f];
        } else if (!CONT_ONLY) {
          const int64_t row = ids[f - Cf] + L.fm_cate_offset;
          if (row < L.n_rows && row_ok(row, L.zero_row0)) {
            atomicAdd(a.g_first + row, dzb * a.w_head[f]);
            a.touched[row] = 1;
          }
        }
      }
    }
    if (CONT_ONLY) continue;
    // deep lookups
    const float* gx = a.dx0 + (int64_t)b * L.dx0_ld + L.dx0_cat_col;
    for (int f0 = 0; f0 < S; f0 += RPI) {
      const int f = f0 + r;
      if (f < S) {
        const int64_t row = ids[f] + L.deep_cate_offset;
        if (row < L.n_rows && row_ok(row, L.zero_row0)) {
          atomicAdd(a.g_table + row * E + d, gx[f * E + d]);
          if (d == 0) a.touched[row] = 1;
        }
      }
    }
  }

  if (Cf > 0) {
    // block reduction of the hot rows -> cont_slab[block][Cf*(E+1)]
    __shared__ float red[4][kMaxHotCont * (E + 1)];   // 8.7 KB at E = 16: LDS does not cap the occupancy
    const int width = Cf * (E + 1);
#pragma unroll
    for (int p = 0; p < NCP; ++p) {
      const int f = p * RPI + r;
      if (p * RPI < Cf && f < Cf) red[wid][f * E + d] = gc[p];
    }
    if (lane < Cf) red[wid][Cf * E + lane] = g1c;
    __syncthreads();
    for (int k = threadIdx.x; k < width; k += blockDim.x)
      a.cont_slab[(int64_t)blockIdx.x * width + k] = red[0][k] + red[1][k] + red[2][k] + red[3][k];
  }
}

// The FM cont-field rows every sample hits, alone (the sorted / lazy backward does the
// rest): E / 4 lanes per sample, one float4 of the dims each, every field of the sample in
// the lane's registers, so a wave covers 64 / (E / 4) samples per load round trip instead
// of one.  Per-element terms as embed_bwd_kernel's; block partials to cont_slab[block].
template <int E, int NC>
__global__ __launch_bounds__(256) void cont_bwd_kernel(EmbBwdArgs a) {
  constexpr int QPR = E / 4, SPW = 64 / QPR;
  const dl_emb_layout& L = a.L;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int q = lane % QPR;
  const int Cf = L.cont_fields;
  const int F = Cf + L.cate_fields + L.fm_extra;
  const float w0 = a.w_head[F + 4 * q], w1 = a.w_head[F + 4 * q + 1];
  const float w2 = a.w_head[F + 4 * q + 2], w3 = a.w_head[F + 4 * q + 3];
  float4 gc[NC];
  float g1[NC / QPR];
#pragma unroll
  for (int f = 0; f < NC; ++f) gc[f] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int j = 0; j < NC / QPR; ++j) g1[j] = 0.f;
  // the butterfly below is the costly part (ds_bpermute), so the samples are dealt to the
  // first `active` blocks, four wave iterations each; the rest write zero slabs
  const int active = min((int)gridDim.x, max(1, (L.batch + 16 * SPW - 1) / (16 * SPW)));
  const int nw = active * (blockDim.x >> 6);
  // the cont rows (the same for every sample) and their first-order head weights, once
  float4 er[NC];
  float wf[NC / QPR];
#pragma unroll
  for (int f = 0; f < NC; ++f) {
    const int64_t row = L.fm_cont_offset + f;
    er[f] = (f < Cf && row_ok(row, L.zero_row0))
                ? *reinterpret_cast<const float4*>(a.table + (L.cont_rows_compact ? f : row) * E + 4 * q)
                : make_float4(0.f, 0.f, 0.f, 0.f);
  }
#pragma unroll
  for (int j = 0; j < NC / QPR; ++j) wf[j] = q + QPR * j < Cf ? a.w_head[q + QPR * j] : 0.f;
  // kIt of the wave's samples loaded together (one memory round trip: at one wave a SIMD the
  // loop is latency-bound), then summed in the same sample order as one at a time
  constexpr int kIt = NC > 16 ? 1 : 4;   // (32 cont rows: one at a time, or the registers spill)
  const int stride = nw * SPW;
  for (int b0 = blockIdx.x < active ? ((blockIdx.x * blockDim.x + threadIdx.x) >> 6) * SPW + lane / QPR : L.batch;
       b0 < L.batch; b0 += kIt * stride) {
    float dzv[kIt], cv[kIt][NC];
    float4 sdv[kIt];
#pragma unroll
    for (int i = 0; i < kIt; ++i) {
      const int b = b0 + i * stride;
      const int bc = b < L.batch ? b : b0;
      dzv[i] = a.dz[bc];
      sdv[i] = *reinterpret_cast<const float4*>(a.fm_sum + (int64_t)bc * E + 4 * q);
#pragma unroll
      for (int f = 0; f < NC; ++f) cv[i][f] = f < Cf ? a.cont[(int64_t)bc * Cf + f] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < kIt; ++i) {
      if (b0 + i * stride >= L.batch) break;
      const float dzb = dzv[i];
      const float4 sd = sdv[i];
      const float d0 = dzb * w0, d1 = dzb * w1, d2 = dzb * w2, d3 = dzb * w3;
#pragma unroll
      for (int f = 0; f < NC; ++f) {
        if (f < Cf) {
          const int64_t row = L.fm_cont_offset + f;
          const float val = cv[i][f];
          float4 e = make_float4(0.f, 0.f, 0.f, 0.f);
          if (row_ok(row, L.zero_row0)) {
            e = er[f];
            e.x *= val; e.y *= val; e.z *= val; e.w *= val;
          }
          gc[f].x += val * d0 * (sd.x - e.x); gc[f].y += val * d1 * (sd.y - e.y);
          gc[f].z += val * d2 * (sd.z - e.z); gc[f].w += val * d3 * (sd.w - e.w);
        }
      }
#pragma unroll
      for (int j = 0; j < NC / QPR; ++j) {
        const int f = q + QPR * j;
        float cf = cv[i][QPR * j];   // cv[i][f] by constant indices (q selects): no scratch
#pragma unroll
        for (int t = 1; t < QPR; ++t)
          if (q == t) cf = cv[i][QPR * j + t];
        if (f < Cf) g1[j] += dzb * wf[j] * cf;
      }
    }
  }
  // the wave's SPW samples (lanes with the same q) summed by butterfly
#pragma unroll
  for (int o = QPR; o < 64; o <<= 1) {
#pragma unroll
    for (int f = 0; f < NC; ++f) {
      if (f < Cf) {
        gc[f].x += __shfl_xor(gc[f].x, o, 64); gc[f].y += __shfl_xor(gc[f].y, o, 64);
        gc[f].z += __shfl_xor(gc[f].z, o, 64); gc[f].w += __shfl_xor(gc[f].w, o, 64);
      }
    }
#pragma unroll
    for (int j = 0; j < NC / QPR; ++j) g1[j] += __shfl_xor(g1[j], o, 64);
  }
  __shared__ __align__(16) float red[4][NC * (E + 1)];
  if (lane < QPR) {
#pragma unroll
    for (int f = 0; f < NC; ++f)
      if (f < Cf) *reinterpret_cast<float4*>(&red[wid][f * E + 4 * q]) = gc[f];
#pragma unroll
    for (int j = 0; j < NC / QPR; ++j)
      if (q + QPR * j < Cf) red[wid][Cf * E + q + QPR * j] = g1[j];
  }
  __syncthreads();
  const int width = Cf * (E + 1);
  for (int k = threadIdx.x; k < width; k += blockDim.x)
    a.cont_slab[(int64_t)blockIdx.x * width + k] = red[0][k] + red[1][k] + red[2][k] + red[3][k];
}

// Folds the cont-field partial slabs into the dense gradient tables.
__global__ __launch_bounds__(256) void cont_reduce_kernel(dl_emb_layout L, const float* slab,
                                                          int blocks, float* g_table,
                                                          float* g_first, uint8_t* touched) {
  const int E = L.emb_dim, Cf = L.cont_fields;
  const int width = Cf * (E + 1);
  const int k = blockIdx.x;
  if (k >= width) return;
  float acc = 0.f;
  for (int t = threadIdx.x; t < blocks; t += blockDim.x) acc += slab[(int64_t)t * width + k];
  acc = wave_sum(acc);
  __shared__ float part[4];
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float tot = part[0] + part[1] + part[2] + part[3];
    int64_t row;
    // compact: the gradients of the C cont rows are a [C] buffer (the record/sharded paths)
    if (k < Cf * E) {
      row = L.fm_cont_offset + k / E;
      if (!row_ok(row, L.zero_row0)) return;
      if (L.cont_rows_compact) row = k / E;
      g_table[row * E + (k % E)] += tot;
    } else {
      row = L.fm_cont_offset + (k - Cf * E);
      if (!row_ok(row, L.zero_row0)) return;
      if (L.cont_rows_compact) row = k - Cf * E;
      g_first[row] += tot;
    }
    touched[row] = 1;
  }
}

// ---------------------------------------------------------------------------
// multi-hot nonzero-mean pooling (deepfm_multi_cate.py:71-111)

struct PoolArgs {
  dl_emb_layout L;
  const int32_t* inv;      // indexed mode (records): row of multi ref = inv_base + inv[b*ns + mb + l]
  int inv_base;
  const float* table;
  const float* first_order;
  const int64_t* ids;
  int ids_col;
  const int32_t* slot_start;
  const int32_t* slot_end;
  int n_slots;
  int fm_col;
  float* x0;
  float* fm_out;
  float* cnt_emb;
  float* cnt_first;
  int32_t* err;
  const float* vals;       // weighted mode: value of multi position l of sample b = vals[b*vals_ld + l]
  int vals_ld;
  // staged mode (IDX; after dl_rec_gather_scatter with multi-hot staging): the row of multi
  // position l of sample b is table row b * multi_width + l (written there by the gather),
  // a position without a row (inv < 0: padding) none
  int staged;
};

// One wave per sample.  A slot's positions are resolved 64 at a time, one per lane (ids or
// the batch index: one coalesced load), then handed to the row loads by __shfl — the
// 64/RPI row loads of a chunk are independent, so they are in flight together instead
// of each waiting on its own id load.  Summation order (per lane, then the xor tree) is
// the same for both modes and for any chunking: dense and record paths pool identically.
// WT (dnn_multi_textline.py:94-103): each row is scaled by its position's value before the
// sum, while the count still tests the unscaled row (count_nonzero of the plain lookup).
template <int E, bool IDX, bool WT = false>
__global__ __launch_bounds__(256) void pool_fwd_kernel(PoolArgs a) {
  constexpr int LPR = E / 4;
  constexpr int RPI = 64 / LPR;
  const dl_emb_layout& L = a.L;
  const int lane = threadIdx.x & 63;
  const int r = lane / LPR, q = lane % LPR;
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int nwaves = (gridDim.x * blockDim.x) >> 6;
  const float4* tab4 = reinterpret_cast<const float4*>(a.table);
  const int ns = index_slots(L), mb = index_multi_base(L);
  for (int b = wave; b < L.batch; b += nwaves) {
    const int64_t* ids = IDX ? nullptr : a.ids + (int64_t)b * L.cate_ld + a.ids_col;
    const int32_t* invb = IDX ? a.inv + (int64_t)b * ns + mb : nullptr;
    const float* valb = WT ? a.vals + (int64_t)b * a.vals_ld : nullptr;
    for (int m = 0; m < a.n_slots; ++m) {
      const int s0 = a.slot_start[m], s1 = a.slot_end[m];
      float4 s = f4_zero();
      float cnt = 0.f, s1v = 0.f, c1 = 0.f;
      for (int c0 = s0; c0 < s1; c0 += 64) {
        const int nl = min(64, s1 - c0);
        // source row of position c0 + lane (-1: padding / zero row)
        long long src = -1;
        float wv = 0.f;
        if (WT && lane < nl) wv = valb[c0 + lane];
        if (lane < nl) {
          if (IDX) {
            const int ri = invb[c0 + lane];
            src = ri < 0 ? -1 : a.staged ? (long long)b * L.multi_width + c0 + lane : (long long)a.inv_base + ri;
          } else {
            const int64_t row = checked_row(ids[c0 + lane], 0, L.n_rows, a.err);
            src = row_ok(row, L.zero_row0) ? row : -1;
          }
        }
        if (a.first_order) {
          const float w = src >= 0 ? (DL_POOL_DIAG_NO_W1 ? 1.f : a.first_order[src]) : 0.f;
          s1v += w;
          c1 += (w != 0.f) ? 1.f : 0.f;
        }
#pragma unroll
        for (int it = 0; it < 64 / RPI; ++it) {
          const int pl = it * RPI + r;
          const long long row = __shfl(src, pl, 64);
          float4 e = f4_zero();
          if (pl < nl && row >= 0) e = tab4[row * LPR + q];
          // tf.reduce_sum(emb, axis=2) then count_nonzero over the slot
          float rs = (e.x + e.y) + (e.z + e.w);
#pragma unroll
          for (int o = 1; o < LPR; o <<= 1) rs += __shfl_xor(rs, o, 64);
          if (q == 0 && pl < nl && rs != 0.f) cnt += 1.f;
          if (WT) {
            const float w = __shfl(wv, pl, 64);
            e.x *= w; e.y *= w; e.z *= w; e.w *= w;   // tf.multiply(emb, value), then the sum
          }
          s.x += e.x; s.y += e.y; s.z += e.z; s.w += e.w;
        }
      }
#pragma unroll
      for (int o = LPR; o < 64; o <<= 1) {
        s.x += __shfl_xor(s.x, o, 64); s.y += __shfl_xor(s.y, o, 64);
        s.z += __shfl_xor(s.z, o, 64); s.w += __shfl_xor(s.w, o, 64);
      }
      cnt = wave_sum(cnt);
      if (r == 0) {
        float4 o4 = f4_zero();
        if (cnt > 0.f) { o4.x = s.x / cnt; o4.y = s.y / cnt; o4.z = s.z / cnt; o4.w = s.w / cnt; }
        *reinterpret_cast<float4*>(a.x0 + (int64_t)b * L.x0_ld + L.x0_pool_col + m * E + 4 * q) = o4;
      }
      if (lane == 0) a.cnt_emb[(int64_t)b * a.n_slots + m] = cnt;
      if (a.first_order) {
        s1v = wave_sum(s1v);
        c1 = wave_sum(c1);
        if (lane == 0) {
          a.fm_out[(int64_t)b * L.fm_ld + a.fm_col + m] = c1 > 0.f ? s1v / c1 : 0.f;
          a.cnt_first[(int64_t)b * a.n_slots + m] = c1;
        }
      }
    }
  }
}

// Ballot-compacted pooling (the default; pool_fwd_kernel above serves more than kPoolMaxSlots
// slots or a multi block wider than kSlotLutMax).  One wave per sample walks the sample's whole
// multi block 64 positions at a time: each lane resolves its position's slot (an LDS table) and
// source row, a __ballot of the valid ones (a row present, not padding, not the zero row) and
// the lane's prefix popcount (mbcnt) give every valid position a compacted queue index, and the
// wave appends (row, slot, value) there in LDS.  Each full queue of 64 is drained 16 rows per
// round with all four rounds' row and first-order loads in flight together: the wave loads only
// the rows the sample references — padding costs no iteration and no predicated-off lanes —
// and every slot's rows are in flight at once instead of slot after slot.  Per-slot sums stay in
// registers (a lane's rows in queue order, then the xor tree over the 16 row groups): the
// order depends only on the positions, so the dense, indexed and staged modes pool identically.
// deepfm_multi_cate.py:73-78: cnt = count_nonzero(reduce_sum(V[ids], axis=2)) per slot,
// out = div_no_nan(reduce_sum(V[ids], axis=1), cnt); the first-order weights likewise.
constexpr int kPoolMaxSlots = 8;
constexpr int kPoolQ = 64;   // compacted rows per drain

template <int E, bool IDX, bool WT>
__global__ __launch_bounds__(256) void pool_fwd_compact_kernel(PoolArgs a) {
  constexpr int LPR = E / 4, RPI = 64 / LPR, NIT = kPoolQ / RPI;
  const dl_emb_layout& L = a.L;
  __shared__ unsigned char lut[kSlotLutMax];
  __shared__ int q_src[4][2 * kPoolQ];
  __shared__ unsigned char q_slot[4][2 * kPoolQ];
  __shared__ float q_val[4][WT ? 2 * kPoolQ : 1];
  const int M = a.n_slots;
  int W = 0;
  for (int m = 0; m < M; ++m) W = max(W, a.slot_end[m]);
  const bool use_lut = W <= kSlotLutMax;
  for (int l = threadIdx.x; use_lut && l < W; l += blockDim.x) {
    int m = 0;
    while (m < M && !(l >= a.slot_start[m] && l < a.slot_end[m])) ++m;
    lut[l] = (unsigned char)m;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int r = lane / LPR, q = lane % LPR;
  int* qs = q_src[wv];
  unsigned char* qm = q_slot[wv];
  float* qv = q_val[wv];
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int nwaves = (gridDim.x * blockDim.x) >> 6;
  const float4* tab4 = reinterpret_cast<const float4*>(a.table);
  const int ns = index_slots(L), mb = index_multi_base(L);
  const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
  for (int b = wave; b < L.batch; b += nwaves) {
    const int64_t* ids = IDX ? nullptr : a.ids + (int64_t)b * L.cate_ld + a.ids_col;
    const int32_t* invb = IDX ? a.inv + (int64_t)b * ns + mb : nullptr;
    const float* valb = WT ? a.vals + (int64_t)b * a.vals_ld : nullptr;
    float4 s[kPoolMaxSlots];
    float cnt[kPoolMaxSlots], s1[kPoolMaxSlots], c1[kPoolMaxSlots];
#pragma unroll
    for (int m = 0; m < kPoolMaxSlots; ++m) { s[m] = f4_zero(); cnt[m] = s1[m] = c1[m] = 0.f; }
    int qn = 0;
    // one drain: queue entries [0, n) (n <= kPoolQ), four rounds of RPI rows, loads first
    auto drain = [&](int n) {
      float4 e[NIT];
      float w[NIT];
      int mm[NIT];
#pragma unroll
      for (int it = 0; it < NIT; ++it) {
        const int j = it * RPI + r;
        const bool in = j < n;
        const int src = in ? qs[j] : -1;
        mm[it] = in ? qm[j] : kPoolMaxSlots;
        e[it] = src >= 0 ? tab4[(long long)((DL_POOL_DIAG & 1) ? 0 : src) * LPR + q] : f4_zero();
        w[it] = (a.first_order && src >= 0 && q == 0) ? (DL_POOL_DIAG_NO_W1 ? 1.f : a.first_order[src]) : 0.f;
      }
#pragma unroll
      for (int it = 0; it < NIT; ++it) {
        float4 x = e[it];
        float rs = (x.x + x.y) + (x.z + x.w);   // tf.reduce_sum(emb, axis=2): the count's test
#pragma unroll
        for (int o = 1; o < LPR; o <<= 1) rs += __shfl_xor(rs, o, 64);
        if (WT) {
          const float vv = (it * RPI + r) < n ? qv[it * RPI + r] : 0.f;
          x.x *= vv; x.y *= vv; x.z *= vv; x.w *= vv;   // tf.multiply(emb, value), then the sum
        }
#pragma unroll
        for (int m = 0; m < kPoolMaxSlots; ++m) {
          if (mm[it] == m) {
            s[m].x += x.x; s[m].y += x.y; s[m].z += x.z; s[m].w += x.w;
            if (q == 0) {
              cnt[m] += rs != 0.f ? 1.f : 0.f;
              s1[m] += w[it];
              c1[m] += w[it] != 0.f ? 1.f : 0.f;
            }
          }
        }
      }
    };
    for (int p0 = 0; p0 < W; p0 += 64) {
      const int pos = p0 + lane;
      int src = -1, m = M;
      float vv = 0.f;
      if (pos < W) {
        if (use_lut) {
          m = lut[pos];
        } else {
          m = 0;
          while (m < M && !(pos >= a.slot_start[m] && pos < a.slot_end[m])) ++m;
        }
        if (m < M) {
          if (IDX) {
            const int ri = invb[pos];
            src = ri < 0 ? -1 : a.staged ? b * L.multi_width + pos : a.inv_base + ri;
          } else {
            const int64_t row = checked_row(ids[pos], 0, L.n_rows, a.err);
            src = row_ok(row, L.zero_row0) ? (int)row : -1;
          }
          if (WT) vv = valb[pos];
        }
      }
      const uint64_t vm = __ballot(src >= 0);
      if (src >= 0) {
        const int c = qn + __popcll(vm & below);
        qs[c] = src;
        qm[c] = (unsigned char)m;
        if (WT) qv[c] = vv;
      }
      qn += __popcll(vm);
      __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): the queue writes landed for the wave
      __builtin_amdgcn_wave_barrier();
      if (qn >= kPoolQ) {
        drain(kPoolQ);
        qn -= kPoolQ;
        __builtin_amdgcn_wave_barrier();
        if (lane < qn) {   // carry the overflow to the queue's front
          qs[lane] = qs[kPoolQ + lane];
          qm[lane] = qm[kPoolQ + lane];
          if (WT) qv[lane] = qv[kPoolQ + lane];
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
      }
    }
    if (qn > 0) drain(qn);
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int m = 0; m < kPoolMaxSlots; ++m) {
      if (m >= M) break;
      float4 t = s[m];
#pragma unroll
      for (int o = LPR; o < 64; o <<= 1) {
        t.x += __shfl_xor(t.x, o, 64); t.y += __shfl_xor(t.y, o, 64);
        t.z += __shfl_xor(t.z, o, 64); t.w += __shfl_xor(t.w, o, 64);
      }
      const float cn = wave_sum(cnt[m]);
      if (DL_POOL_DIAG & 2) {   // diagnostics: no output stores (one lane keeps the sums live)
        const float sv = wave_sum(s1[m]);
        if (t.x + cn + sv == 1234.5f) a.x0[0] = t.y;
        continue;
      }
      if (r == 0) {
        float4 o4 = f4_zero();
        if (cn > 0.f) { o4.x = t.x / cn; o4.y = t.y / cn; o4.z = t.z / cn; o4.w = t.w / cn; }
        *reinterpret_cast<float4*>(a.x0 + (int64_t)b * L.x0_ld + L.x0_pool_col + m * E + 4 * q) = o4;
      }
      if (lane == 0) a.cnt_emb[(int64_t)b * M + m] = cn;
      if (a.first_order) {
        const float sv = wave_sum(s1[m]), cc = wave_sum(c1[m]);
        if (lane == 0) {
          a.fm_out[(int64_t)b * L.fm_ld + a.fm_col + m] = cc > 0.f ? sv / cc : 0.f;
          a.cnt_first[(int64_t)b * M + m] = cc;
        }
      }
    }
  }
}

// compacted pooling when the slots fit (n_slots <= kPoolMaxSlots; width checked on the host)
#ifndef DL_POOL_COMPACT
#define DL_POOL_COMPACT 1
#endif

struct PoolBwdArgs {
  dl_emb_layout L;
  const int64_t* ids;
  int ids_col;
  const int32_t* slot_start;
  const int32_t* slot_end;
  int n_slots;
  int fm_col;
  const float* x0;
  const float* fm_sum;
  const float* dz;
  const float* w_head;
  const float* dx0;
  int dx0_pool_col;
  const float* cnt_emb;
  const float* cnt_first;
  float* g_table;
  float* g_first;
  uint8_t* touched;
  const float* vals;       // weighted mode (see PoolArgs)
  int vals_ld;
};

template <int E, bool WT = false>
__global__ __launch_bounds__(256) void pool_bwd_kernel(PoolBwdArgs a) {
  constexpr int RPI = 64 / E;
  const dl_emb_layout& L = a.L;
  const int lane = threadIdx.x & 63;
  const int r = lane / E, d = lane % E;
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int nwaves = (gridDim.x * blockDim.x) >> 6;
  const int F = (L.fm_cont ? L.cont_fields : 0) + L.cate_fields + L.fm_extra;
  for (int b = wave; b < L.batch; b += nwaves) {
    const int64_t* ids = a.ids + (int64_t)b * L.cate_ld + a.ids_col;
    const float dzb = L.use_fm ? a.dz[b] : 0.f;
    const float dsec = L.use_fm ? dzb * a.w_head[F + d] : 0.f;
    const float sd = L.use_fm ? a.fm_sum[(int64_t)b * E + d] : 0.f;
    for (int m = 0; m < a.n_slots; ++m) {
      const int s0 = a.slot_start[m], s1 = a.slot_end[m];
      const float pooled = a.x0[(int64_t)b * L.x0_ld + L.x0_pool_col + m * E + d];
      float dp = a.dx0[(int64_t)b * L.dx0_ld + a.dx0_pool_col + m * E + d];
      if (L.use_fm) dp += dsec * (sd - pooled);
      const float c = a.cnt_emb[(int64_t)b * a.n_slots + m];
      const float gv = c > 0.f ? dp / c : 0.f;   // div_no_nan gradient
      for (int l0 = s0; l0 < s1; l0 += RPI) {
        const int l = l0 + r;
        if (l < s1) {
          const int64_t row = ids[l];
          if (row < L.n_rows && row_ok(row, L.zero_row0)) {
            atomicAdd(a.g_table + row * E + d, WT ? gv * a.vals[(int64_t)b * a.vals_ld + l] : gv);
            if (d == 0) a.touched[row] = 1;
          }
        }
      }
      if (L.use_fm && a.g_first) {
        const float c1 = a.cnt_first[(int64_t)b * a.n_slots + m];
        const float g1 = c1 > 0.f ? dzb * a.w_head[a.fm_col + m] / c1 : 0.f;
        for (int l = s0 + lane; l < s1; l += 64) {
          const int64_t row = ids[l];
          if (row < L.n_rows && row_ok(row, L.zero_row0)) {
            atomicAdd(a.g_first + row, g1);
            a.touched[row] = 1;
          }
        }
      }
    }
  }
}

// no_cat_ok: x0_cat_col == -1 accepted (the plain table and the indexed lookups: the single-cate
// embeddings are then not written, dl_gemm_s3_nt_gather reads them from the table or the
// compact rows itself)
static int check_layout(const dl_emb_layout* L, bool no_cat_ok = false) {
  DL_CHECK_ARG(L != nullptr, "layout is NULL");
  const int E = L->emb_dim;
  DL_CHECK_ARG(E == 4 || E == 8 || E == 16 || E == 32 || E == 64, "emb_dim %d not in {4,8,16,32,64}", E);
  DL_CHECK_ARG(L->batch >= 0 && L->n_rows > 0, "bad batch/n_rows");
  DL_CHECK_ARG(L->x0_ld % 4 == 0 && (L->x0_cat_col % 4 == 0 || (no_cat_ok && L->x0_cat_col == -1)),
               "x0_ld and x0_cat_col must be multiples of 4");
  DL_CHECK_ARG(!L->x0_bf16 || L->fm_extra == 0, "bf16 x0 needs fm_extra == 0 (pooled vectors are read as f32)");
  DL_CHECK_ARG(!L->fm_extra || L->x0_pool_col % 4 == 0, "x0_pool_col must be a multiple of 4");
  DL_CHECK_ARG(L->cont_fields <= kMaxHotCont || !(L->use_fm && L->fm_cont),
               "at most %d FM cont fields", kMaxHotCont);
  return 0;
}

static int emb_grid(int B) {
  int g = (B + 3) / 4;
  if (g > 4096) g = 4096;
  return g < 1 ? 1 : g;
}

}  // namespace dl

using namespace dl;

template <int REC>
static int launch_embed_fwd(const dl_emb_layout* L, const EmbArgs& a, void* stream);

extern "C" int dl_embed_fwd(const dl_emb_layout* L, const float* table, const float* first_order,
                            const int64_t* cate, const float* cont, const float* vector,
                            float* x0, float* fm_out, float* fm_sum, int32_t* err, void* stream) {
  if (int rc = check_layout(L, true)) return rc;
  DL_CHECK_ARG(table && cate && x0, "NULL table/cate/x0");
  DL_CHECK_ARG(!L->use_fm || (first_order && fm_out && fm_sum), "FM outputs required");
  if (L->batch == 0) return 0;
  EmbArgs a{*L, nullptr, 0, table, first_order, cate, cont, vector, x0, fm_out, fm_sum, err};
  return launch_embed_fwd<0>(L, a, stream);
}

extern "C" int dl_embed_fwd_slots(const dl_emb_layout* L, const float* slots, const int64_t* cate, const float* cont,
                                  const float* vector, float* x0, float* fm_out, float* fm_sum, int32_t* err,
                                  void* stream) {
  if (int rc = check_layout(L, true)) return rc;
  DL_CHECK_ARG(slots && cate && x0, "NULL slots/cate/x0");
  DL_CHECK_ARG(!L->use_fm || (fm_out && fm_sum), "FM outputs required");
  DL_CHECK_ARG((uintptr_t)slots % 16 == 0, "the slot plane must be 16-B aligned");
  if (L->batch == 0) return 0;
  EmbArgs a{*L, nullptr, 0, slots, slots + L->emb_dim, cate, cont, vector, x0, fm_out, fm_sum, err};
  return launch_embed_fwd<3>(L, a, stream);
}

// whether dl_embed_fwd_gtab takes this layout: E = 8 / 16 (the lookup's instantiations with at
// most kGtabMaxNps passes; E = 32 / 64 run one all-slots form) and the FM slots within them
extern "C" int dl_embed_fwd_gtab_ok(const dl_emb_layout* L) {
  if (!L || (L->emb_dim != 8 && L->emb_dim != 16)) return 0;
  const int fs = L->use_fm ? (L->fm_cont ? L->cont_fields : 0) + L->cate_fields : 0;
  const int rpi = 64 / (L->emb_dim / 4);
  return (fs + rpi - 1) / rpi <= kGtabMaxNps ? 1 : 0;
}

extern "C" int dl_embed_fwd_gtab(const dl_emb_layout* L, const float* plane, int32_t slot_plane, const int64_t* cate,
                                 const float* cont, const float* vector, float* x0, float* fm_out, float* fm_sum,
                                 uint32_t* gtab, int32_t* err, void* stream) {
  if (int rc = check_layout(L, true)) return rc;
  DL_CHECK_ARG(plane && cate && gtab, "NULL plane/cate/gtab");
  DL_CHECK_ARG(L->x0_cat_col == -1, "gtab: the deep rows go to the offset table, not x0 (x0_cat_col -1)");
  DL_CHECK_ARG(x0 || (L->x0_cont_col < 0 && L->x0_vec_col < 0), "gtab: x0 columns to write but x0 NULL");
  DL_CHECK_ARG(L->fm_extra == 0 && L->multi_width == 0, "gtab: single-valued fields only");
  DL_CHECK_ARG(!L->use_fm || (slot_plane && fm_out), "gtab: FM models read the slot plane and write fm_out");
  DL_CHECK_ARG((uintptr_t)plane % 16 == 0 && (uintptr_t)gtab % 16 == 0, "gtab: plane / table must be 16-B aligned");
  DL_CHECK_ARG((unsigned long long)L->n_rows * L->emb_dim * (slot_plane ? 8 : 4) < kGtabMasked,
               "gtab: the plane spans past the 32-bit offsets");
  DL_CHECK_ARG(dl_embed_fwd_gtab_ok(L), "gtab: more than %d passes of FM slots a sample", kGtabMaxNps);
  if (L->batch == 0) return 0;
  EmbArgs a{*L, nullptr, 0, plane, slot_plane ? plane + L->emb_dim : nullptr, cate, cont, vector, x0, fm_out, fm_sum,
            err};
  a.gtab = gtab;
  return slot_plane ? launch_embed_fwd<3>(L, a, stream) : launch_embed_fwd<0>(L, a, stream);
}

extern "C" int dl_embed_fwd_indexed(const dl_emb_layout* L, const float* rows, const float* rows_first,
                                    const int32_t* inv, int32_t inv_base, const float* cont, const float* vector,
                                    float* x0, float* fm_out, float* fm_sum, void* stream) {
  if (int rc = check_layout(L, true)) return rc;
  DL_CHECK_ARG(rows && inv && x0, "NULL rows/inv/x0");
  DL_CHECK_ARG(!L->use_fm || (rows_first && fm_out && fm_sum), "FM outputs required");
  if (L->batch == 0) return 0;
  EmbArgs a{*L, inv, inv_base, rows, rows_first, nullptr, cont, vector, x0, fm_out, fm_sum, nullptr};
  return launch_embed_fwd<0>(L, a, stream);
}

extern "C" int dl_embed_fwd_staged(const dl_emb_layout* L, const float* fmst, const float* rows_first,
                                   const int32_t* inv, int32_t n_rep, const float* cont, const float* vector,
                                   float* x0, float* fm_out, float* fm_sum, void* stream) {
  if (int rc = check_layout(L)) return rc;
  DL_CHECK_ARG(inv && x0, "NULL inv/x0");
  DL_CHECK_ARG(!L->use_fm || (fmst && rows_first && fm_out && fm_sum), "FM inputs / outputs required");
  DL_CHECK_ARG(!L->use_fm || !L->fm_cont || L->cont_rows_compact, "the FM cont-field rows come compact");
  if (L->batch == 0) return 0;
  EmbArgs a{*L, inv, n_rep, fmst ? fmst : x0, rows_first, nullptr, cont, vector, x0, fm_out, fm_sum, nullptr};
  a.staged = 1;
  return launch_embed_fwd<0>(L, a, stream);
}

extern "C" int dl_embed_fwd_rec(const dl_emb_layout* L, const float* rec, int32_t rec_ld, int32_t rec_flags,
                                const float* rows_rep, const float* rows_rep1, const int64_t* cate,
                                const float* cont, const float* vector, const float* hist, int32_t hist_len,
                                const float* opt, int32_t lag, float* x0, float* fm_out, float* fm_sum,
                                int32_t* err, void* stream) {
  const int32_t has_first = rec_flags & DL_REC_FIRST;
  if (int rc = check_layout(L)) return rc;
  DL_CHECK_ARG(rec && cate && x0 && hist && opt, "NULL argument");
  DL_CHECK_ARG(hist_len >= 2 && hist_len <= 8192 && (hist_len & (hist_len - 1)) == 0,
               "hist_len must be a power of two in [2, 8192] (the ring is staged in LDS)");
  DL_CHECK_ARG(rec_ld % 4 == 0 && rec_ld >= 3 * L->emb_dim + 4, "rec_ld %d too small", rec_ld);
  DL_CHECK_ARG(L->multi_width == 0 && L->fm_extra == 0, "record forward: single-valued fields only");
  const int Cf = (L->use_fm && L->fm_cont) ? L->cont_fields : 0;
  DL_CHECK_ARG(Cf == 0 || (L->cont_rows_compact && rows_rep && (!has_first || rows_rep1)),
               "the FM cont-field rows come compact in rows_rep / rows_rep1");
  DL_CHECK_ARG(!L->use_fm || (fm_out && fm_sum && Cf + L->cate_fields <= 64), "FM outputs required (<= 64 fields)");
  if (L->batch == 0) return 0;
  EmbArgs a{*L, nullptr, 0, rows_rep, rows_rep1, cate, cont, vector, x0, fm_out, fm_sum, err,
            rec, make_rec_cfg(L->emb_dim, rec_ld, rec_flags, hist_len), hist, opt, lag};
  return launch_embed_fwd<1>(L, a, stream);
}

extern "C" int dl_embed_fwd_rec_flat(const dl_emb_layout* L, const float* rec, int32_t rec_ld, int32_t rec_flags,
                                     const float* rows_rep, const float* rows_rep1, const int64_t* cate,
                                     const float* cont, const float* vector, const float* opt, float* x0,
                                     float* fm_out, float* fm_sum, int32_t* err, void* stream) {
  const int32_t has_first = rec_flags & DL_REC_FIRST;
  if (int rc = check_layout(L)) return rc;
  DL_CHECK_ARG(rec && cate && x0 && opt, "NULL argument");
  DL_CHECK_ARG(rec_ld % 4 == 0 && rec_ld >= 3 * L->emb_dim + 4, "rec_ld %d too small", rec_ld);
  DL_CHECK_ARG(L->multi_width == 0 && L->fm_extra == 0, "record forward: single-valued fields only");
  const int Cf = (L->use_fm && L->fm_cont) ? L->cont_fields : 0;
  DL_CHECK_ARG(Cf == 0 || (L->cont_rows_compact && rows_rep && (!has_first || rows_rep1)),
               "the FM cont-field rows come compact in rows_rep / rows_rep1");
  DL_CHECK_ARG(!L->use_fm || (fm_out && fm_sum && Cf + L->cate_fields <= 64), "FM outputs required (<= 64 fields)");
  if (L->batch == 0) return 0;
  EmbArgs a{*L, nullptr, 0, rows_rep, rows_rep1, cate, cont, vector, x0, fm_out, fm_sum, err,
            rec, make_rec_cfg(L->emb_dim, rec_ld, rec_flags, 2), nullptr, opt, 0};
  return launch_embed_fwd<2>(L, a, stream);
}

template <int REC>
static int launch_embed_fwd(const dl_emb_layout* L, const EmbArgs& a, void* stream) {
  DL_CHECK_ARG((L->use_fm ? (L->fm_cont ? L->cont_fields : 0) + 2 * L->cate_fields : L->cate_fields) <= kMaxSlots,
               "too many fields per sample for the gather kernel (max %d slots)", kMaxSlots);
  const int tiles = (L->batch + kTileSamples - 1) / kTileSamples;
  const int gmax = REC == 1 ? 1024 : 8192;   // record mode: each block stages the alpha ring once
  const dim3 grid(tiles < gmax ? tiles : gmax), block(256);
  const int nslot = (L->use_fm ? (L->fm_cont ? L->cont_fields : 0) + L->cate_fields : 0) +
                    (L->x0_cat_col >= 0 ? L->cate_fields : 0);
  const int rpi = 64 / (L->emb_dim / 4);
  const int nps = nslot > 0 ? (nslot + rpi - 1) / rpi : 1;
  const size_t lds = REC == 1 ? (size_t)(a.rc.hist_mask + 1) * sizeof(float) : 0;
  hipStream_t st = as_stream(stream);
#define DL_FWD(E_, N_) hipLaunchKernelGGL((embed_fwd_kernel<E_, N_, REC>), grid, block, lds, st, a)
  switch (L->emb_dim) {
    case 16:
      switch (nps) {
        case 1: DL_FWD(16, 1); break; case 2: DL_FWD(16, 2); break; case 3: DL_FWD(16, 3); break;
        case 4: DL_FWD(16, 4); break; case 5: DL_FWD(16, 5); break; case 6: DL_FWD(16, 6); break;
        case 7: DL_FWD(16, 7); break; default: DL_FWD(16, 8); break;
      }
      break;
    case 8:
      switch (nps) {
        case 1: DL_FWD(8, 1); break; case 2: DL_FWD(8, 2); break; case 3: DL_FWD(8, 3); break;
        default: DL_FWD(8, 4); break;
      }
      break;
    case 4: DL_FWD(4, 2); break;
    case 32: DL_FWD(32, 16); break;
    case 64: DL_FWD(64, 32); break;
  }
#undef DL_FWD
  DL_RETURN_LAUNCH("dl_embed_fwd");
}

extern "C" int dl_embed_bwd_grid(const dl_emb_layout* L) { return emb_grid(L->batch) < 1024 ? emb_grid(L->batch) : 1024; }

extern "C" int dl_embed_bwd(const dl_emb_layout* L, const float* table, const int64_t* cate,
                            const float* cont, const float* dz, const float* w_head,
                            const float* fm_sum, const float* dx0, float* g_table, float* g_first,
                            uint8_t* touched, float* cont_slab, int32_t cont_slab_blocks,
                            void* stream) {
  if (int rc = check_layout(L)) return rc;
  if (L->batch == 0) return 0;
  const int grid = dl_embed_bwd_grid(L);
  const bool hot = L->use_fm && L->fm_cont && L->cont_fields > 0;
  DL_CHECK_ARG(!hot || (cont_slab && cont_slab_blocks >= grid), "cont_slab needs %d blocks", grid);
  DL_CHECK_ARG(!L->use_fm || (dz && w_head && fm_sum && g_first), "FM backward inputs required");
  EmbBwdArgs a{*L, table, cate, cont, dz, w_head, fm_sum, dx0, g_table, g_first, touched, cont_slab};
  DL_DISPATCH_E(L->emb_dim, hipLaunchKernelGGL((embed_bwd_kernel<kE, false>), dim3(grid), dim3(256), 0,
                                               as_stream(stream), a));
  DL_RETURN_LAUNCH("dl_embed_bwd");
}

extern "C" int dl_embed_cont_reduce(const dl_emb_layout* L, const float* cont_slab, int32_t blocks,
                                    float* g_table, float* g_first, uint8_t* touched, void* stream) {
  if (int rc = check_layout(L)) return rc;
  if (!(L->use_fm && L->fm_cont && L->cont_fields > 0)) return 0;
  const int width = L->cont_fields * (L->emb_dim + 1);
  hipLaunchKernelGGL(cont_reduce_kernel, dim3(width), dim3(256), 0, as_stream(stream), *L,
                     cont_slab, blocks, g_table, g_first, touched);
  DL_RETURN_LAUNCH("dl_embed_cont_reduce");
}

extern "C" int dl_pool_fwd(const dl_emb_layout* L, const float* table, const float* first_order,
                           const int64_t* ids, int32_t ids_col, const int32_t* slot_start,
                           const int32_t* slot_end, int32_t n_slots, int32_t fm_col, float* x0,
                           float* fm_out, float* cnt_emb, float* cnt_first, int32_t* err,
                           void* stream) {
  if (int rc = check_layout(L)) return rc;
  DL_CHECK_ARG(n_slots >= 0 && slot_start && slot_end, "bad slots");
  DL_CHECK_ARG(!first_order || (fm_out && cnt_first), "first-order pooling needs fm_out/cnt_first");
  if (L->batch == 0 || n_slots == 0) return 0;
  PoolArgs a{*L, nullptr, 0, table, first_order, ids, ids_col, slot_start, slot_end, n_slots, fm_col,
             x0, fm_out, cnt_emb, cnt_first, err, nullptr, 0};
  if (DL_POOL_COMPACT && n_slots <= kPoolMaxSlots)
    DL_DISPATCH_E(L->emb_dim, hipLaunchKernelGGL((pool_fwd_compact_kernel<kE, false, false>), dim3(emb_grid(L->batch)),
                                                 dim3(256), 0, as_stream(stream), a))
  else DL_DISPATCH_E(L->emb_dim, hipLaunchKernelGGL((pool_fwd_kernel<kE, false>), dim3(emb_grid(L->batch)),
                                               dim3(256), 0, as_stream(stream), a));
  DL_RETURN_LAUNCH("dl_pool_fwd");
}

extern "C" int dl_pool_fwd_indexed(const dl_emb_layout* L, const float* rows, const float* rows_first,
                                   const int32_t* inv, int32_t inv_base, const int32_t* slot_start,
                                   const int32_t* slot_end, int32_t n_slots, int32_t fm_col, float* x0,
                                   float* fm_out, float* cnt_emb, float* cnt_first, void* stream) {
  if (int rc = check_layout(L)) return rc;
  DL_CHECK_ARG(rows && inv && x0 && cnt_emb && slot_start && slot_end && n_slots >= 0, "NULL argument");
  DL_CHECK_ARG(L->multi_width > 0, "indexed pooling needs the multi-hot refs in the index (multi_width)");
  DL_CHECK_ARG(!rows_first || (fm_out && cnt_first), "first-order pooling needs fm_out/cnt_first");
  if (L->batch == 0 || n_slots == 0) return 0;
  PoolArgs a{*L, inv, inv_base, rows, rows_first, nullptr, 0, slot_start, slot_end, n_slots, fm_col,
             x0, fm_out, cnt_emb, cnt_first, nullptr, nullptr, 0};
  if (DL_POOL_COMPACT && n_slots <= kPoolMaxSlots)
    DL_DISPATCH_E(L->emb_dim, hipLaunchKernelGGL((pool_fwd_compact_kernel<kE, true, false>), dim3(emb_grid(L->batch)),
                                                 dim3(256), 0, as_stream(stream), a))
  else DL_DISPATCH_E(L->emb_dim, hipLaunchKernelGGL((pool_fwd_kernel<kE, true>), dim3(emb_grid(L->batch)),
                                               dim3(256), 0, as_stream(stream), a));
  DL_RETURN_LAUNCH("dl_pool_fwd_indexed");
}

extern "C" int dl_pool_fwd_staged(const dl_emb_layout* L, const float* mst, const float* mst1, const int32_t* inv,
                                  const int32_t* slot_start, const int32_t* slot_end, int32_t n_slots, int32_t fm_col,
                                  float* x0, float* fm_out, float* cnt_emb, float* cnt_first, void* stream) {
  if (int rc = check_layout(L)) return rc;
  DL_CHECK_ARG(mst && inv && x0 && cnt_emb && slot_start && slot_end && n_slots >= 0, "NULL argument");
  DL_CHECK_ARG(L->multi_width > 0, "staged pooling needs the multi-hot refs in the index (multi_width)");
  DL_CHECK_ARG(!mst1 || (fm_out && cnt_first), "first-order pooling needs fm_out/cnt_first");
  if (L->batch == 0 || n_slots == 0) return 0;
  PoolArgs a{*L, inv, 0, mst, mst1, nullptr, 0, slot_start, slot_end, n_slots, fm_col,
             x0, fm_out, cnt_emb, cnt_first, nullptr, nullptr, 0};
  a.staged = 1;
  if (DL_POOL_COMPACT && n_slots <= kPoolMaxSlots)
    DL_DISPATCH_E(L->emb_dim, hipLaunchKernelGGL((pool_fwd_compact_kernel<kE, true, false>), dim3(emb_grid(L->batch)),
                                                 dim3(256), 0, as_stream(stream), a))
  else DL_DISPATCH_E(L->emb_dim, hipLaunchKernelGGL((pool_fwd_kernel<kE, true>), dim3(emb_grid(L->batch)),
                                               dim3(256), 0, as_stream(stream), a));
  DL_RETURN_LAUNCH("dl_pool_fwd_staged");
}

extern "C" int dl_pool_bwd(const dl_emb_layout* L, const int64_t* ids, int32_t ids_col,
                           const int32_t* slot_start, const int32_t* slot_end, int32_t n_slots,
                           int32_t fm_col, const float* x0, const float* fm_sum, const float* dz,
                           const float* w_head, const float* dx0, int32_t dx0_pool_col,
                           const float* cnt_emb, const float* cnt_first, float* g_table,
                           float* g_first, uint8_t* touched, void* stream) {
  if (int rc = check_layout(L)) return rc;
  if (L->batch == 0 || n_slots == 0) return 0;
  PoolBwdArgs a{*L, ids, ids_col, slot_start, slot_end, n_slots, fm_col, x0, fm_sum, dz, w_head,
                dx0, dx0_pool_col, cnt_emb, cnt_first, g_table, g_first, touched, nullptr, 0};
  DL_DISPATCH_E(L->emb_dim, hipLaunchKernelGGL(pool_bwd_kernel<kE>, dim3(emb_grid(L->batch)),
                                               dim3(256), 0, as_stream(stream), a));
  DL_RETURN_LAUNCH("dl_pool_bwd");
}

extern "C" int dl_pool_fwd_weighted(const dl_emb_layout* L, const float* table, const int64_t* ids,
                                    int32_t ids_col, const float* values, int32_t values_ld,
                                    const int32_t* slot_start, const int32_t* slot_end, int32_t n_slots,
                                    float* x0, float* cnt_emb, int32_t* err, void* stream) {
  if (int rc = check_layout(L)) return rc;
  DL_CHECK_ARG(table && ids && values && x0 && cnt_emb && slot_start && slot_end && n_slots >= 0,
               "NULL argument");
  DL_CHECK_ARG(values_ld >= 0, "bad values_ld");
  DL_CHECK_ARG(L->x0_pool_col % 4 == 0, "x0_pool_col must be a multiple of 4");
  if (L->batch == 0 || n_slots == 0) return 0;
  PoolArgs a{*L, nullptr, 0, table, nullptr, ids, ids_col, slot_start, slot_end, n_slots, 0,
             x0, nullptr, cnt_emb, nullptr, err, values, values_ld};
  if (DL_POOL_COMPACT && n_slots <= kPoolMaxSlots)
    DL_DISPATCH_E(L->emb_dim, hipLaunchKernelGGL((pool_fwd_compact_kernel<kE, false, true>), dim3(emb_grid(L->batch)),
                                                 dim3(256), 0, as_stream(stream), a))
  else DL_DISPATCH_E(L->emb_dim, hipLaunchKernelGGL((pool_fwd_kernel<kE, false, true>), dim3(emb_grid(L->batch)),
                                               dim3(256), 0, as_stream(stream), a));
  DL_RETURN_LAUNCH("dl_pool_fwd_weighted");
}

extern "C" int dl_pool_bwd_weighted(const dl_emb_layout* L, const int64_t* ids, int32_t ids_col,
                                    const float* values, int32_t values_ld, const int32_t* slot_start,
                                    const int32_t* slot_end, int32_t n_slots, const float* dx0,
                                    int32_t dx0_pool_col, const float* cnt_emb, float* g_table,
                                    uint8_t* touched, void* stream) {
  if (int rc = check_layout(L)) return rc;
  DL_CHECK_ARG(!L->use_fm, "weighted pooling is a deep-only lookup (dnn_multi_textline.py:94-103)");
  DL_CHECK_ARG(ids && values && dx0 && cnt_emb && g_table && touched && slot_start && slot_end,
               "NULL argument");
  if (L->batch == 0 || n_slots == 0) return 0;
  PoolBwdArgs a{*L, ids, ids_col, slot_start, slot_end, n_slots, 0, nullptr, nullptr, nullptr, nullptr,
                dx0, dx0_pool_col, cnt_emb, nullptr, g_table, nullptr, touched, values, values_ld};
  DL_DISPATCH_E(L->emb_dim, hipLaunchKernelGGL((pool_bwd_kernel<kE, true>), dim3(emb_grid(L->batch)),
                                               dim3(256), 0, as_stream(stream), a));
  DL_RETURN_LAUNCH("dl_pool_bwd_weighted");
}

// ---------------------------------------------------------------------------
// Deterministic backward from the batch index (index.hip): one group of E lanes
// per unique row sums its references in sorted order.  For FM references
//   d/dV[row] = dsec_b * (fm_sum_b - V[row])   (d second / d e_f, value 1)
// so a row's FM part is  sum_b dsec_b*fm_sum_b - V[row] * sum_b dsec_b.

namespace dl {

struct BwdSortedArgs {
  dl_emb_layout L;
  const float* table;      // local table (single GPU) or NULL
  const float* rows_u;     // gathered rows per unique id [u][E] (sharded) or NULL
  const uint32_t* uniq;
  const int32_t* seg_off;
  const int32_t* n_uniq;
  const int32_t* refs;
  int world;
  const float* dz;
  const float* w_head;
  const float* fm_sum;
  const float* dx0;
  float* g_out;
  float* g1_out;
  uint8_t* touched;
  int compact;
  const int32_t* upos;     // compact: the slot of unique row u in rows_u / g_out (sharded exchange
                           // blocks, dl_shard_route; -1 = no slot), NULL = u itself
};


// One unique row's gradient from its segment sums, to g_out (compact: by unique index).
template <int E>
__device__ __forceinline__ void embed_bwd_sorted_row(const BwdSortedArgs& a, long long u, int q, const SegGrad4& sgr) {
  const dl_emb_layout& L = a.L;
  const int64_t row = decode_key(a.uniq[u], a.world);
  if (row < 0 || row >= L.n_rows) return;
  const long long slot = a.upos ? (long long)a.upos[u] : u;
  if (slot < 0) return;
  float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
  if (sgr.dsum.x != 0.f || sgr.dsum.y != 0.f || sgr.dsum.z != 0.f || sgr.dsum.w != 0.f)
    v = *reinterpret_cast<const float4*>((a.rows_u ? a.rows_u + slot * E : a.table + row * E) + 4 * q);
  float4 g;
  g.x = seg_row_grad(sgr.s.x, sgr.dsum.x, sgr.x.x, sgr.dsum.x != 0.f ? v.x : 0.f);
  g.y = seg_row_grad(sgr.s.y, sgr.dsum.y, sgr.x.y, sgr.dsum.y != 0.f ? v.y : 0.f);
  g.z = seg_row_grad(sgr.s.z, sgr.dsum.z, sgr.x.z, sgr.dsum.z != 0.f ? v.z : 0.f);
  g.w = seg_row_grad(sgr.s.w, sgr.dsum.w, sgr.x.w, sgr.dsum.w != 0.f ? v.w : 0.f);
  const long long o = a.compact ? slot : row;
  *reinterpret_cast<float4*>(a.g_out + o * E + 4 * q) = g;
  if (q == 0) {
    if (a.g1_out && (a.compact || L.use_fm)) a.g1_out[o] = sgr.g1;
    if (!a.compact) a.touched[row] = 1;
  }
}

// float4 lanes (E/4 per unique row, as rec_bwd_adam_kernel): a wave keeps 64/(E/4)
// rows' segment walks in flight; sums are bit-identical to the per-dim form.
template <int E>
__global__ __launch_bounds__(256) void embed_bwd_sorted_kernel(BwdSortedArgs a) {
  constexpr int LPR = E / 4;
  const dl_emb_layout& L = a.L;
  const long long gt = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const int q = (int)(gt % LPR);
  const long long group0 = gt / LPR, ngroups = (long long)gridDim.x * blockDim.x / LPR;
  const int S = L.cate_fields;
  const int ns = index_slots(L);
  const int Cf = (L.use_fm && L.fm_cont) ? L.cont_fields : 0;
  const int F = Cf + S + L.fm_extra;
  const long long nrefs = (long long)L.batch * ns;
  const int nu = clamp_uniq(a.n_uniq, nrefs);
  const float* ws = a.w_head + F + 4 * q;   // not 16-B aligned
  const float4 wsec = L.use_fm ? make_float4(ws[0], ws[1], ws[2], ws[3]) : make_float4(0.f, 0.f, 0.f, 0.f);
  const SegGradIn sg{L, a.seg_off, a.refs, a.dz, a.w_head, a.fm_sum, a.dx0};
  for (long long u = group0; u < nu; u += ngroups) {
    const SegRange cr = seg_range(sg, u, nu, nrefs);
    if (cr.e1 - cr.e0 > kSegLong) continue;   // a hot row: embed_bwd_long_kernel
    const SegGrad4 sgr = segment_grad4_range<E>(sg, cr.e0, cr.e1, -2, q, nrefs, wsec);
    embed_bwd_sorted_row<E>(a, u, q, sgr);
  }
}

template <int E>
__global__ __launch_bounds__(256) void embed_bwd_long_kernel(BwdSortedArgs a) {
  __shared__ SegLongLds sh;
  const dl_emb_layout& L = a.L;
  const int q = threadIdx.x % (E / 4);
  const int S = L.cate_fields, ns = index_slots(L);
  const int Cf = (L.use_fm && L.fm_cont) ? L.cont_fields : 0;
  const int F = Cf + S + L.fm_extra;
  const long long nrefs = (long long)L.batch * ns;
  const int nu = clamp_uniq(a.n_uniq, nrefs);
  const float* ws = a.w_head + F + 4 * q;
  const float4 wsec = L.use_fm ? make_float4(ws[0], ws[1], ws[2], ws[3]) : make_float4(0.f, 0.f, 0.f, 0.f);
  const SegGradIn sg{L, a.seg_off, a.refs, a.dz, a.w_head, a.fm_sum, a.dx0};
  for_long_segments<E>(sg, nu, nrefs, wsec, sh, [&](long long u, const SegGrad4& s) { embed_bwd_sorted_row<E>(a, u, q, s); });
}

}  // namespace dl

extern "C" int dl_embed_bwd_sorted(const dl_emb_layout* L, const float* table, const float* rows_u,
                                   const uint32_t* uniq_keys, const int32_t* seg_off, const int32_t* n_uniq,
                                   const int32_t* sorted_refs, int32_t world, int64_t max_uniq,
                                   const float* dz, const float* w_head, const float* fm_sum,
                                   const float* dx0, float* g_out, float* g1_out, uint8_t* touched,
                                   int32_t compact, const int32_t* upos, void* stream) {
  if (int rc = check_layout(L)) return rc;
  DL_CHECK_ARG(uniq_keys && seg_off && n_uniq && sorted_refs && dx0 && g_out, "NULL argument");
  DL_CHECK_ARG(table || rows_u, "need the table or the gathered rows");
  DL_CHECK_ARG(compact || touched, "dense output needs the touched flags");
  DL_CHECK_ARG(!L->use_fm || (dz && w_head && fm_sum), "FM backward inputs required");
  if (max_uniq <= 0) return 0;
  DL_CHECK_ARG(L->dx0_ld % 4 == 0 && L->dx0_cat_col % 4 == 0, "dx0 must be float4 aligned");
  long long blocks = (max_uniq * (L->emb_dim / 4) + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  BwdSortedArgs a{*L, table, rows_u, uniq_keys, seg_off, n_uniq, sorted_refs, world, dz, w_head, fm_sum, dx0,
                  g_out, g1_out, touched, compact, compact ? upos : nullptr};
  DL_DISPATCH_E(L->emb_dim, {
    hipLaunchKernelGGL(embed_bwd_sorted_kernel<kE>, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), a);
    hipLaunchKernelGGL(embed_bwd_long_kernel<kE>, dim3(1024), dim3(256), 0, as_stream(stream), a);
  });
  DL_RETURN_LAUNCH("dl_embed_bwd_sorted");
}

extern "C" int dl_embed_cont_bwd(const dl_emb_layout* L, const float* table, const float* cont,
                                 const float* dz, const float* w_head, const float* fm_sum, float* cont_slab,
                                 int32_t cont_slab_blocks, void* stream) {
  if (int rc = check_layout(L)) return rc;
  if (L->batch == 0 || !(L->use_fm && L->fm_cont && L->cont_fields > 0)) return 0;
  // blocks: cont_slab_blocks, at most dl_embed_bwd_grid (blocks past the samples' share write
  // zero partials, so a caller may pass just the blocks that hold samples: same partials)
  const int grid = min(dl_embed_bwd_grid(L), (int)cont_slab_blocks);
  DL_CHECK_ARG(cont_slab && cont_slab_blocks >= 1, "cont_slab needs at least one block");
  EmbBwdArgs a{*L, table, nullptr, cont, dz, w_head, fm_sum, nullptr, nullptr, nullptr, nullptr, cont_slab};
  DL_DISPATCH_E(L->emb_dim, {
    if (L->cont_fields <= 16)
      hipLaunchKernelGGL((cont_bwd_kernel<kE, 16>), dim3(grid), dim3(256), 0, as_stream(stream), a);
    else
      hipLaunchKernelGGL((cont_bwd_kernel<kE, kMaxHotCont>), dim3(grid), dim3(256), 0, as_stream(stream), a);
  });
  DL_RETURN_LAUNCH("dl_embed_cont_bwd");
}
