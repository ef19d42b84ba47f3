// fp32 tower GEMMs on the bf16 matrix cores, three-plane split ("s3").
//
// Every f32 x splits exactly into three bf16 planes, x = hi + mid + lo:
//   hi = rn_bf16(x), mid = rn_bf16(x - hi), lo = rn_bf16(x - hi - mid)
// (x - hi is exact in f32 and spans <= 16 significant bits, x - hi - mid <= 8, so lo is
// exact: a lossless 6-byte encoding of a normal f32).  A product a.b is then
//   hi.hi + hi.mid + mid.hi + mid.mid + hi.lo + lo.hi        (dropped: mid.lo, lo.mid, lo.lo)
// with each bf16 x bf16 product exact in the f32 accumulator of v_mfma_f32_16x16x32_bf16;
// the dropped terms are <= 2^-25 |a.b|, below one f32 rounding.  Six bf16 MFMAs (6 x 16
// cycles) replace the eight f32 v_mfma_f32_16x16x4_f32 (8 x 32 cycles) of a 32-deep k
// step: the f32 products of deepfm_pipeline.py:150-152 and their gradients at f32
// accuracy (tests: fp64 reference, relative error <= 2e-6) at up to 2.7x the f32 rate.
//
// Products (all operands f32 in HBM; the split happens in registers):
//   NT  C[M][N] = A[M][K] . B[N][K]^T   forward (B = W^T) and dX (B = W): A streamed
//       from HBM straight into MFMA fragments and split in registers; B pre-split into
//       planes (dl_split3, the weights: a few hundred KB) staged through LDS per 32-deep
//       k chunk.  Block 256 x 208 (8 waves x 32 rows x 13 column fragments).
//   TN  C[M][N] = sum_k X[k][M] Y[k][N]  weight gradients, split-K slabs over the batch:
//       both operands batch-major f32, split into planes on their way into LDS, read back as
//       MFMA fragments by CDNA4's transposing ds_read_b64_tr_b16.  Block 128 x 416
//       (8 waves x 32 rows x 13 column fragments).
#include "common.h"
#include <cstdlib>
#include <type_traits>

namespace dl {

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef unsigned int s3_u32x4_t __attribute__((__vector_size__(4 * sizeof(unsigned int))));
typedef short shortx8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float floatx2_t __attribute__((ext_vector_type(2)));
typedef __attribute__((__vector_size__(4 * sizeof(__fp16)))) __fp16 s3_fp16x4_t;

// two f32 -> packed bf16 (v_cvt_pk_bf16_f32, round to nearest even; element 0 low)
__device__ __forceinline__ uint32_t pk_bf16(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((floatx2_t){a, b}, bf16x2_t));
}

// planes of two consecutive elements
__device__ __forceinline__ void split2(float x0, float x1, uint32_t& h, uint32_t& m, uint32_t& l) {
#pragma clang fp contract(off)
  h = pk_bf16(x0, x1);
  const float r0 = x0 - __uint_as_float(h << 16), r1 = x1 - __uint_as_float(h & 0xffff0000u);
  m = pk_bf16(r0, r1);
  const float s0 = r0 - __uint_as_float(m << 16), s1 = r1 - __uint_as_float(m & 0xffff0000u);
  l = pk_bf16(s0, s1);
}

// 8 consecutive f32 (two float4) -> the three 8 x bf16 MFMA operands
__device__ __forceinline__ void split8(const float4& a, const float4& b, shortx8& h, shortx8& m, shortx8& l) {
  uint4 H, M, L;
  split2(a.x, a.y, H.x, M.x, L.x);
  split2(a.z, a.w, H.y, M.y, L.y);
  split2(b.x, b.y, H.z, M.z, L.z);
  split2(b.z, b.w, H.w, M.w, L.w);
  h = __builtin_bit_cast(shortx8, H);
  m = __builtin_bit_cast(shortx8, M);
  l = __builtin_bit_cast(shortx8, L);
}

// acc += a.b over the six significant plane products (small terms first)
__device__ __forceinline__ floatx4 mfma_s3(const shortx8& ah, const shortx8& am, const shortx8& al,
                                           const shortx8& bh, const shortx8& bm, const shortx8& bl,
                                           floatx4 acc) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, bm, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, bh, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bm, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, acc, 0, 0, 0);
  return acc;
}

// The same six products, each with the operands' roles swapped (B's planes as the MFMA's src A):
// the accumulator then holds C^T's 16 x 16 block — lane (kq, cl) has row cl, columns 4kq .. 4kq + 3
// — so the NT epilogue stores a float4 of one output row per lane straight from registers.
__device__ __forceinline__ floatx4 mfma_s3_t(const shortx8& ah, const shortx8& am, const shortx8& al,
                                             const shortx8& bh, const shortx8& bm, const shortx8& bl,
                                             floatx4 acc) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bh, al, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bl, ah, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bm, am, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bh, am, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bm, ah, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bh, ah, acc, 0, 0, 0);
  return acc;
}

__device__ __forceinline__ int s3_xcd_tile(int bid, int T) {
  const int x = bid & 7;
  const int q = T >> 3, rm = T & 7;
  return (x < rm ? x * (q + 1) : rm * (q + 1) + (x - rm) * q) + (bid >> 3);
}

struct S3Params {
  const float* A;
  const void* B;
  float* C;
  const float* mask;
  int M, N, K;
  int lda, ldb, ldc, ldm;
  long long b_plane;         // NT: elements between the planes of B
  int k_per_split;           // TN
  long long c_split_stride;  // TN
  uint16_t* bits;            // NT: the ReLU sign bitmask [M][ldbits] (written by S3_RELU, read by S3_MASKBITS)
  int ldbits;
  // NT gather (dl_gemm_s3_nt_gather): A's columns [0, 32 g_chunks) are the embedding rows of
  // the row's ids (row ids[m][f] + id_off, f = k >> g_esh, column k & (2^g_esh - 1)), read
  // straight from the table G (g_ld floats a row; a masked or invalid row reads as zeros)
  const float* G;
  const int64_t* ids;
  const int32_t* ids32;      // (training form) int32 row indices instead of ids: < 0 = the zero row
  float* a_store;            // (training form) the gathered columns also written here (x0, ld lda)
  long long id_off, n_rows;
  int ids_ld, g_ld, g_fields, g_esh, g_chunks, zero_row0;
  unsigned g_bytes;          // G's buffer range (bytes, < 0xFFFFFF00: the masked rows' offset)
  // (the table form, dl_gemm_s3_nt_gather_tab) the rows' byte offsets already resolved by the
  // lookup (common.h kGtab*): the block stages its part of the table as it stands
  const uint32_t* gofs;
};

// S3_MASKBITS: the ReluGrad mask from the forward's bitmask (bit c & 15 of halfword
// [row][c >> 4] = h[row][c] > 0) instead of the f32 activations — 1/32 of the mask bytes
enum { S3_STORE = 0, S3_RELU = 1, S3_MASK = 2, S3_MASKBITS = 3 };

#ifndef DL_S3_MWLATE
#define DL_S3_MWLATE 1   // dX bitmask words loaded before the last k step (0: before the main loop)
#endif
#ifndef DL_S3_GDIAG
#define DL_S3_GDIAG 0   // diagnostics build: the gathered A rows all read table row 0 (timing only)
#endif
#ifndef DL_S3_BPF
#define DL_S3_BPF 0   // 1: NT pins the next fragment's weight reads ahead of this one's MFMAs
#endif                // (sched_barrier; measured slower than leaving the order to the scheduler)

#ifndef DL_S3_PF
#define DL_S3_PF 1    // NT: weight fragments read this many fragments ahead of their MFMAs
#endif
#ifndef DL_S3_SGB
#define DL_S3_SGB 0   // NT: pin the order (fragment f + PF's LDS reads, then fragment f's 12 MFMAs)
#endif                // with sched_group_barrier, so the reads are not sunk next to their use

#ifndef DL_S3_ASMB
#define DL_S3_ASMB 0  // NT: the weight fragments' LDS reads as inline asm, DL_S3_PF fragments ahead,
#endif                // each fragment's MFMAs behind a hand-counted lgkmcnt wait tied to its registers

#ifndef DL_S3_ESPLIT
#define DL_S3_ESPLIT 1   // NT: chunk c + 1's A planes split in the middle of chunk c's MFMAs
                         // (fwd_l1 114.7 -> 110.9 us alone, profiles/r05f/s3_ab.txt)
#endif
#ifndef DL_S3_ESASM
#define DL_S3_ESASM 1   // early-split step: weight fragment reads as asm, DL_S3_ES_PF fragments ahead
#endif
#ifndef DL_S3_ES_PF
#define DL_S3_ES_PF 2
#endif

#ifndef DL_S3_TNSTAG
#define DL_S3_TNSTAG 0   // TN2: waves 4-7 split + store the next step's tiles BEFORE their MFMAs
#endif                   // (waves 0-3 after), so the two waves of a SIMD overlap VALU/LDS with MFMA

#ifndef DL_S3_TN2
#define DL_S3_TN2 1   // weight gradients: the double-buffered TN kernel (0: the single-buffer one)
#endif

#ifndef DL_S3_DIAG
#define DL_S3_DIAG 0   // diagnostics builds: 1 = no epilogue stores, 2 = no MFMAs either;
                       // 3 = no stores, no A loads (constant A); 4 = no stores, no B LDS reads;
                       // 5 = no stores, no per-chunk barrier; 6 = no plane split (A in NT, both
                       // operands in TN2: the f32 bits taken as planes); 7 = NT A pieces at k = 32c + 4kq
                       // and + 16 (results wrong: timing only)
#endif

// ---------------------------------------------------------------------------- NT
// B chunk images: per plane 208 rows x 32 k (64 B), 16-B piece kq of row j at slot
// kq ^ ((j >> 2) & 2): conflict-free fragment reads for ds_read_b128's four lane groups
// ({0-3,12-15,20-27}, {4-11,16-19,28-31}, ... MI355X_MICROARCH.md §LDS; found by exhaustive
// search over per-row slot permutations), filled by LDS-DMA
// (global_load_lds_dwordx4: one instruction = 16 rows) two chunks ahead into a ring of three
// buffers, so no chunk waits a full memory round trip for its weights.
constexpr int kNtBM = 256, kNtBN = 208, kNtNF = 13;
constexpr int kNtPlane = kNtBN * 32;                             // bf16 elements of one plane image
constexpr int kNtBuf = 3 * kNtPlane;
constexpr int kNtDma = 3 * kNtBN / 16;                           // DMA instructions per chunk (39)
constexpr int kNtDmaW = (kNtDma + 7) / 8;                        // per wave (5)
constexpr size_t kNtLds = 3 * kNtBuf * sizeof(unsigned short);  // 119,808 B
constexpr int kNtEP = kNtBN + 4;                                 // epilogue tile pitch (floats)
static_assert(8 * 16 * kNtEP * sizeof(float) <= kNtLds, "epilogue tiles fit the ring");
// NT gather: the block's row offsets into G, one u32 per (field, row) after the ring, fields
// kNtGfs words apart (272 = 16 mod 64 banks: the 2-4 fields a wave instruction reads fall in
// disjoint banks); at most kNtGmaxF fields within 160 KB of LDS
constexpr int kNtGfs = 272;
constexpr int kNtGmaxF = (160 * 1024 - (int)kNtLds) / (kNtGfs * 4);
constexpr uint32_t kNtGmasked = 0xFFFFFF00u;
static_assert(kNtBM == kGtabRows && kNtGfs == kGtabPitch && kNtGmasked == kGtabMasked,
              "the lookup's offset table is the block's LDS table as it stands");

__device__ __forceinline__ int nt_slot(int j, int kq) { return kq ^ ((j >> 2) & 2); }   // an involution in kq

// One weight fragment's three plane reads (planes kNtPlane apart = 13,312 B), issued as asm
// so the compiler cannot sink them next to their MFMAs; lds_wait<N> then waits until at most
// N LDS reads are outstanding (LDS reads complete in order) and ties the fragment's registers
// to that wait, so its MFMAs cannot be scheduled above it.
__device__ __forceinline__ void nt_rd3(uint32_t a, shortx8& h, shortx8& m, shortx8& l) {
  asm volatile("ds_read_b128 %0, %3\n\tds_read_b128 %1, %3 offset:13312\n\tds_read_b128 %2, %3 offset:26624"
               : "=&v"(h), "=&v"(m), "=&v"(l)
               : "v"(a)
               : "memory");
}
#define DL_LDS_WAIT(N, h, m, l) asm volatile("s_waitcnt lgkmcnt(" #N ")" : "+v"(h), "+v"(m), "+v"(l))

// s_waitcnt vmcnt(n) (n < 64), other counters untouched
#define DL_WAIT_VMCNT(n) __builtin_amdgcn_s_waitcnt(((n) & 0xF) | (((n) >> 4) << 14) | (0x7 << 4) | (0xF << 8))

// DIRECT: the transposed accumulator layout (mfma_s3_t) and the epilogue straight from registers
// — one 16-B store of four consecutive columns per lane and fragment (a wave instruction writes
// 16 rows x 64 B), ReLU / ReluGrad bitmask in registers — instead of the transpose through the
// LDS ring; the bitmask words the dX epilogue needs are loaded before the main loop.  Needs
// N % 4 == 0, ldc % 4 == 0 and an even ldbits (the host picks it then; otherwise the LDS form).
// GATHER: the embedding-lookup fusion of the flushed-table forward (dl_gemm_s3_nt_gather): the
// first 32 g_chunks columns of A are fetched row by row from the table through the ids (an 8-float
// piece never straddles two rows: E % 8 == 0), the rest from A as usual.  The values are the
// ones the lookup would have written to A (a copy), so C is bit-identical to the unfused pair.
// STORE_A (with GATHER: the training form): the column-tile-0 blocks also write the gathered A
// pieces into p.a_store (x0) as they split them, for the weight gradient that streams x0 later —
// four 16-B stores a lane and step, past the range (dropped) where there is nothing to write,
// so every wave's vector-memory queue keeps one straight-line count.
template <int EPI, bool DIRECT = false, bool GATHER = false, bool STORE_A = false>
__global__ __launch_bounds__(512) void gemm_s3_nt_kernel(S3Params p) {
  extern __shared__ __attribute__((aligned(16))) unsigned short lds[];   // [3 bufs][3 planes][BN][32]
  constexpr int NW = 8, BM = kNtBM, DMAW = kNtDmaW;
  const unsigned short* __restrict__ Bp = reinterpret_cast<const unsigned short*>(p.B);
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ntm = (p.M + BM - 1) / BM, ntn = (p.N + kNtBN - 1) / kNtBN;
  const int t = s3_xcd_tile(blockIdx.x, ntm * ntn);
  const int i0 = (t / ntn) * BM, j0 = (t % ntn) * kNtBN;
  const int cl = lane & 15, kq = lane >> 4;
  const int r0 = i0 + wid * 32;
  const bool ok0 = r0 + cl < p.M, ok1 = r0 + 16 + cl < p.M;
  // rows as float4 arrays (16-B aligned: A is, and lda % 4 == 0); loads are unconditional from
  // clamped addresses, and out-of-range pieces are zeroed afterwards (no exec-masked loads)
  // byte offsets of this lane's rows (the host checks M * lda * 4 < 2^31)
  const uint32_t a_off0 = 4u * (uint32_t)(min(r0 + cl, p.M - 1) * p.lda);
  const uint32_t a_off1 = 4u * (uint32_t)(min(r0 + 16 + cl, p.M - 1) * p.lda);
  const auto a_rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)p.A, (short)0, p.M * p.lda * 4, 0x00020000);
  const int KC = (p.K + 31) / 32;

  // LDS-DMA of chunk c into buffer `buf`: instruction g (g = wid, wid + 8, ...) fills plane
  // g / 13, rows 16 (g % 13) .. +16; lane L writes slot L & 3 of row L >> 2 and so fetches
  // the piece that belongs there.  Rows past N / k past K read clamped in-range data (their
  // products are discarded / multiplied by A's zeros).
  // The DMA is inline asm: hipcc tracks a builtin LDS-DMA as a pending LDS write and then
  // waits vmcnt(0) before the first use of any load it tracks (the A loads), draining the
  // whole prefetch every chunk.  Invisible to its bookkeeping, the DMA is counted by hand in
  // publish() below; hipcc's own waits for the A loads count only those (over-waiting, safe).
  const uint32_t lds_base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) unsigned short*)lds;
  // Every wave issues exactly kNtDmaW instructions (the last one clamped: wave 7 repeats
  // instruction kNtDma - 1, the same bytes to the same place), so the vmcnt bookkeeping below
  // is one straight-line count for every wave and the compiler's own waits can count too.
  // Addressing: a scalar base per instruction (plane, first row of its 16) and one 32-bit
  // lane offset per chunk (row within the 16, k piece) shared by all of a wave's instructions,
  // so the prefetch holds one VGPR rather than a 64-bit address per instruction.
  auto dma_b = [&](int c, int buf) {
    const uint32_t vk = 2u * (uint32_t)min(32 * c + 8 * nt_slot(lane >> 2, lane & 3), p.K - 8);
    const uint32_t vrow = vk + 2u * (uint32_t)((lane >> 2) * p.ldb);
    int lim = p.N - 1 - j0;   // opaque per call: the rows past N's offsets are not hoisted
    asm volatile("" : "+s"(lim));
#pragma unroll
    for (int i = 0; i < DMAW; ++i) {
      const int g = min(wid + NW * i, kNtDma - 1);
      const int pl = g / 13, rb = 16 * (g % 13);
      const int rbase = j0 + min(rb, lim);
      // rows past N read row N - 1 (their products are discarded)
      const uint32_t voff = rb + 15 <= lim ? vrow : vk + 2u * (uint32_t)(min(lane >> 2, lim - min(rb, lim)) * p.ldb);
      const unsigned short* sb = Bp + pl * p.b_plane + (long long)rbase * p.ldb;
      const uint32_t dst = lds_base + 2u * (uint32_t)(buf * kNtBuf + pl * kNtPlane + rb * 32);
      unsigned keep;
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
                   : "=&s"(keep) : "v"(voff), "s"(sb), "s"(__builtin_amdgcn_readfirstlane(dst)) : "memory");
    }
  };
  // A: this lane's 8 floats of rows r0 + cl, r0 + 16 + cl at k = 32c + 8kq
  // A through a buffer descriptor: a piece outside M or K gets an offset past the descriptor's
  // range and reads as zeros, so no fixup follows a load (overwriting a register whose load
  // is in flight would cost a wait for it).
  uint32_t* gtab = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(lds) + kNtLds);
  const auto g_rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)p.G, (short)0, (int)p.g_bytes, 0x00020000);
  auto load_a = [&](int c, float4 (&ra)[4]) {
    if constexpr (GATHER) {
      if (c < p.g_chunks) {   // uniform: the chunk lies in the gathered columns
        const uint32_t em = (1u << p.g_esh) - 1u;
        const int r0l = wid * 32 + cl;
        if (DL_S3_KPERM) {
          // the k-permuted planes: this lane's pieces at k = 32c + 4kq and k + 16 (a wave
          // instruction then reads whole 64-B rows, 16 B a lane): two fields a row for E < 32
          const int ka = 32 * c + 4 * kq, kb = ka + 16;
          const int fa = ka >> p.g_esh, fb = kb >> p.g_esh;
          const uint32_t ca = 4u * ((uint32_t)ka & em), cb = 4u * ((uint32_t)kb & em);
          const uint32_t ta0 = gtab[fa * kNtGfs + r0l], ta1 = gtab[fa * kNtGfs + r0l + 16];
          const uint32_t tb0 = gtab[fb * kNtGfs + r0l], tb1 = gtab[fb * kNtGfs + r0l + 16];
          const uint32_t a0 = ok0 ? ta0 + ca : kNtGmasked, b0 = ok0 ? tb0 + cb : kNtGmasked;
          const uint32_t a1 = ok1 ? ta1 + ca : kNtGmasked, b1 = ok1 ? tb1 + cb : kNtGmasked;
          ra[0] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(g_rsrc, (int)a0, 0, 0));
          ra[1] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(g_rsrc, (int)b0, 0, 0));
          ra[2] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(g_rsrc, (int)a1, 0, 0));
          ra[3] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(g_rsrc, (int)b1, 0, 0));
        } else {
          // natural order: this lane's 8 floats k = 32c + 8kq .. + 7 of each row lie in one field
          const int k = 32 * c + 8 * kq;
          const int f = k >> p.g_esh;
          const uint32_t col = 4u * ((uint32_t)k & em);
          const uint32_t t0 = gtab[f * kNtGfs + r0l], t1 = gtab[f * kNtGfs + r0l + 16];
          const uint32_t o0 = ok0 ? t0 + col : kNtGmasked, o1 = ok1 ? t1 + col : kNtGmasked;
          ra[0] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(g_rsrc, (int)o0, 0, 0));
          ra[1] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(g_rsrc, (int)(o0 + 16u), 0, 0));
          ra[2] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(g_rsrc, (int)o1, 0, 0));
          ra[3] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(g_rsrc, (int)(o1 + 16u), 0, 0));
        }
        return;
      }
    }
    if (DL_S3_DIAG == 3) {
      ra[0] = ra[1] = ra[2] = ra[3] = make_float4(1.f + c, 2.f, 3.f, 4.f);
      return;
    }
    // DL_S3_KPERM (common.h s3_kpos): a whole chunk's pieces at k = 32c + 4kq and + 16, so
    // each instruction reads one contiguous 64-B half line per row instead of four 16-B pieces
    // of a whole line (DL_S3_DIAG 7: the same loads against natural-order planes, timing only)
    const bool perm = (DL_S3_KPERM || DL_S3_DIAG == 7) && 32 * c + 32 <= p.K;
    const int k = perm ? 32 * c + 4 * kq : 32 * c + 8 * kq;
    const uint32_t d2 = perm ? 64u : 16u;
    const bool kin = k < p.K;
    const uint32_t o0 = ok0 && kin ? a_off0 + 4u * k : 0x80000000u;
    const uint32_t o1 = ok1 && kin ? a_off1 + 4u * k : 0x80000000u;
    ra[0] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(a_rsrc, (int)o0, 0, 0));
    ra[1] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(a_rsrc, (int)(o0 + d2), 0, 0));
    ra[2] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(a_rsrc, (int)o1, 0, 0));
    ra[3] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(a_rsrc, (int)(o1 + d2), 0, 0));
  };

  floatx4 acc[2][kNtNF];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int f = 0; f < kNtNF; ++f) acc[a][f] = floatx4{0.f, 0.f, 0.f, 0.f};

  // DIRECT ReluGrad: this lane's rows' bitmask words for the tile's 13 halfwords (j0 / 16 ..
  // + 12), 7 dwords from the dword holding the first (ldbits even: rows are dword aligned),
  // loaded before the last k chunk's step (load_mw below), so the epilogue does not wait a
  // memory round trip for them and their 14 registers are not held through the main loop
  // (loaded before it they cost 7 spilled VGPRs)
  uint32_t mw[DIRECT && EPI == S3_MASKBITS ? 2 : 1][7];
  auto load_mw = [&]() {
    if constexpr (DIRECT && EPI == S3_MASKBITS) {
#pragma unroll
      for (int a = 0; a < 2; ++a) {
        const int row = min(r0 + 16 * a + cl, p.M - 1);
        const uint32_t* wp = reinterpret_cast<const uint32_t*>(p.bits + (long long)row * p.ldbits) + (j0 >> 5);
#pragma unroll
        for (int i = 0; i < 7; ++i) mw[a][i] = wp[i];
      }
    }
  };
  if (!DL_S3_MWLATE) load_mw();

  float4 raA[4], raB[4];
  // prologue: B chunks 0 and 1 in flight, A chunks 0 and 1
  if constexpr (GATHER) {
    // the weight DMA first, then the block's (field, row) table of row offsets from its ids
    // (coalesced over the id matrix), published by a barrier before any A piece is fetched
    dma_b(0, 0);
    dma_b(1, 1);
    if (!STORE_A && p.gofs) {
      // the table form: the lookup resolved the offsets already, in this table's layout — one
      // contiguous copy (four 16-B pieces a thread in flight: one round trip for 26 fields)
      const uint4* src = reinterpret_cast<const uint4*>(p.gofs + (long long)(i0 / BM) * p.g_fields * kNtGfs);
      uint4* dst = reinterpret_cast<uint4*>(gtab);
      const int n16 = p.g_fields * (kNtGfs / 4);
      for (int b = 0; b < n16; b += 4 * NW * 64) {
        uint4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = src[min(b + u * NW * 64 + tid, n16 - 1)];
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (b + u * NW * 64 + tid < n16) dst[b + u * NW * 64 + tid] = v[u];
      }
    }
    // (eight ids a thread in flight at once: one memory round trip per 4,096 entries; sixteen spill)
    const int tot = !STORE_A && p.gofs ? 0 : BM * p.g_fields;
    constexpr int kGU = 8;
    for (int b = 0; b < tot; b += kGU * NW * 64) {
      long long idv[kGU];
#pragma unroll
      for (int u = 0; u < kGU; ++u) {
        const int i = min(b + u * NW * 64 + tid, tot - 1);
        const int rr = i / p.g_fields, f = i - rr * p.g_fields;
        const long long at = (long long)min(i0 + rr, p.M - 1) * p.ids_ld + f;
        if (STORE_A) {
          const int32_t r32 = p.ids32[at];
          idv[u] = r32 < 0 ? -1 - p.id_off : (long long)r32;   // < 0: below row 0 after the offset
        } else {
          idv[u] = p.ids[at];
        }
      }
#pragma unroll
      for (int u = 0; u < kGU; ++u) {
        const int i = b + u * NW * 64 + tid;
        if (i < tot) {
          const int rr = i / p.g_fields, f = i - rr * p.g_fields;
          const long long id = idv[u] + p.id_off;
          const bool v = id >= 0 && id < p.n_rows && (id > 0 || !p.zero_row0);
          // DL_S3_GDIAG (diagnostics build, wrong results): every valid reference reads row 0
          gtab[f * kNtGfs + rr] = v ? (DL_S3_GDIAG ? 0u : (uint32_t)id * (uint32_t)(4 * p.g_ld)) : kNtGmasked;
        }
      }
    }
    __syncthreads();
    load_a(0, raA);
    load_a(1, raB);
  } else {
  dma_b(0, 0);
  load_a(0, raA);
  dma_b(1, 1);     // unconditional, like every prefetch below: chunks past KC read clamped
  load_a(1, raB);  // weights into a free buffer and zeros for A
  }

  // The per-chunk barrier is a bare s_barrier after explicit counter waits: __syncthreads()
  // carries a workgroup release fence, which the compiler lowers to vmcnt(0) — a wait for
  // every load in flight, including the A loads and weight DMA issued for two chunks ahead,
  // so each chunk paid a full memory round trip.  Here a wave waits only for the batches
  // older than the one it just issued (vmcnt counts in issue order), which include its DMA of
  // the chunk the barrier publishes.
  auto publish = [&](int c) {           // chunk c + 1's weights -> every wave
    if (c + 1 < KC) {
      if (STORE_A) DL_WAIT_VMCNT(DMAW + 8);    // ... and the step's four x0 stores, issued before the DMA
      else DL_WAIT_VMCNT(DMAW + 4);   // every batch but chunk c + 2's: chunk c + 1's DMA too
    }
    else {
      DL_WAIT_VMCNT(0);                   // the epilogue reuses the ring: nothing may still land
    }

    __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): this wave's fragment reads are done
    __builtin_amdgcn_s_barrier();
  };
  // chunk 0's B must have landed
  publish(-1);

#if DL_S3_ESPLIT
  if constexpr (EPI != S3_MASK) {
    // Early split: chunk c + 1's A planes are split in the middle of chunk c's fragments (its
    // MFMAs issue beside the VALU work), so after each barrier the waves start on MFMAs instead of
    // on the split.  Per step c: A(c + 2) into the raw registers chunk c came in (split during
    // step c - 1), fragments 0..kNtEsAt, the split of chunk c + 1 (its wait covers only loads older
    // than A(c + 2)), B(c + 2) by LDS-DMA, the other fragments, the barrier (every batch but
    // A(c + 2) + B(c + 2) landed: chunk c + 1's weights).  Same products in the same order.
    constexpr int kNtEsAt = 6;
    shortx8 pA[6], pB[6];
    auto splitp = [&](float4 (&ra)[4], shortx8 (&P)[6]) {
      split8(ra[0], ra[1], P[0], P[1], P[2]);
      split8(ra[2], ra[3], P[3], P[4], P[5]);
      asm volatile("" : "+v"(P[0]), "+v"(P[1]), "+v"(P[2]), "+v"(P[3]), "+v"(P[4]), "+v"(P[5]));
    };
    // STORE_A: chunk c's raw A pieces into x0 (column-tile-0 blocks, gathered chunks, rows < M)
    const auto st_rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)p.a_store, (short)0, STORE_A ? p.M * p.lda * 4 : 0,
                                                           0x00020000);
    auto store_a = [&](int c, const float4 (&ra)[4]) {
      if constexpr (STORE_A) {
        const bool on = j0 == 0 && c < p.g_chunks;
        const uint32_t k4 = 4u * (uint32_t)(32 * c + 8 * kq);
        const uint32_t o0 = on && ok0 ? a_off0 + k4 : 0x80000000u, o1 = on && ok1 ? a_off1 + k4 : 0x80000000u;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(s3_u32x4_t, ra[0]), st_rsrc, (int)o0, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(s3_u32x4_t, ra[1]), st_rsrc, (int)(o0 + 16u), 0, 0);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(s3_u32x4_t, ra[2]), st_rsrc, (int)o1, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(s3_u32x4_t, ra[3]), st_rsrc, (int)(o1 + 16u), 0, 0);
      }
    };
    splitp(raA, pA);
    store_a(0, raA);
    auto step_es = [&](int c, shortx8 (&P)[6], shortx8 (&Pn)[6], float4 (&R)[4], float4 (&F)[4]) {
      load_a(c + 2, F);
      asm volatile("" ::: "memory");   // the loads issue here, not sunk to the mid-step split
      const uint32_t b_addr = lds_base + 2u * (uint32_t)((c % 3) * kNtBuf + cl * 32 + 8 * nt_slot(cl, kq));
      const unsigned short* Bs = lds + (c % 3) * kNtBuf;
      auto rd_b = [&](int f, shortx8& bh, shortx8& bm, shortx8& bl) {
        const int j = 16 * f + cl;
        const int o = j * 32 + 8 * nt_slot(j, kq);
        bh = *reinterpret_cast<const shortx8*>(&Bs[o]);
        bm = *reinterpret_cast<const shortx8*>(&Bs[kNtPlane + o]);
        bl = *reinterpret_cast<const shortx8*>(&Bs[2 * kNtPlane + o]);
      };
      (void)b_addr;
      (void)rd_b;
      // DL_S3_ESASM: each fragment's three plane reads as asm issued ES_PF fragments ahead, and an
      // lgkmcnt wait tied to its registers right before its MFMAs (hipcc, left alone, issued
      // each pair of fragments' reads just ahead of their MFMAs: the LDS latency in the MFMA
      // stream once a pair); same operands, same order of products
      constexpr int EPF = DL_S3_ESASM ? DL_S3_ES_PF : 1, ENB = EPF + 1;
      shortx8 bb[ENB][3];
#pragma unroll
      for (int i = 0; i < EPF; ++i) {
        if (DL_S3_ESASM) nt_rd3(b_addr + 1024u * i, bb[i][0], bb[i][1], bb[i][2]);
        else rd_b(i, bb[i][0], bb[i][1], bb[i][2]);
      }
#pragma unroll
      for (int f = 0; f < kNtNF; ++f) {
        if (f + EPF < kNtNF) {
          if (DL_S3_ESASM) nt_rd3(b_addr + 1024u * (f + EPF), bb[(f + EPF) % ENB][0], bb[(f + EPF) % ENB][1], bb[(f + EPF) % ENB][2]);
          else rd_b(f + EPF, bb[(f + EPF) % ENB][0], bb[(f + EPF) % ENB][1], bb[(f + EPF) % ENB][2]);
        }
        if (DL_S3_ESASM) {
          shortx8 &h = bb[f % ENB][0], &m = bb[f % ENB][1], &l = bb[f % ENB][2];
          const int younger = min(EPF, kNtNF - 1 - f);   // fragments whose reads follow f's
          if (younger >= 3) DL_LDS_WAIT(9, h, m, l);
          else if (younger == 2) DL_LDS_WAIT(6, h, m, l);
          else if (younger == 1) DL_LDS_WAIT(3, h, m, l);
          else DL_LDS_WAIT(0, h, m, l);
        }
        const shortx8 bh = bb[f % ENB][0], bm = bb[f % ENB][1], bl = bb[f % ENB][2];
        if (DIRECT) {
          acc[0][f] = mfma_s3_t(P[0], P[1], P[2], bh, bm, bl, acc[0][f]);
          acc[1][f] = mfma_s3_t(P[3], P[4], P[5], bh, bm, bl, acc[1][f]);
        } else {
          acc[0][f] = mfma_s3(P[0], P[1], P[2], bh, bm, bl, acc[0][f]);
          acc[1][f] = mfma_s3(P[3], P[4], P[5], bh, bm, bl, acc[1][f]);
        }
        if (f == kNtEsAt) {
          if (c + 1 < KC) splitp(R, Pn);
          store_a(c + 1, R);   // (past KC: chunk KC's pieces fall outside the gathered chunks: dropped)
          dma_b(c + 2, (c + 2) % 3);
        }
      }
      publish(c);
    };
    int c = 0;
    for (; c + 1 < KC; c += 2) {
      step_es(c, pA, pB, raB, raA);
      step_es(c + 1, pB, pA, raA, raB);
    }
    if (DL_S3_MWLATE) load_mw();   // under the peeled last step's MFMAs (odd KC), else before the epilogue
    if (c < KC) step_es(c, pA, pB, raB, raA);
  } else
#endif
  {
  auto step = [&](int c, float4 (&ra)[4]) {
    shortx8 ah[2], am[2], al[2];
    if (DL_S3_DIAG == 6) {   // timing only: the f32 bits taken as planes, no split
      ah[0] = __builtin_bit_cast(shortx8, ra[0]); am[0] = __builtin_bit_cast(shortx8, ra[1]); al[0] = ah[0];
      ah[1] = __builtin_bit_cast(shortx8, ra[2]); am[1] = __builtin_bit_cast(shortx8, ra[3]); al[1] = ah[1];
    } else {
      split8(ra[0], ra[1], ah[0], am[0], al[0]);
      split8(ra[2], ra[3], ah[1], am[1], al[1]);
    }
    // hipcc's wait for chunk c's A counts only its own loads (4 a batch), so it must come
    // before the next batch is issued or it would also wait for part of that batch: the empty
    // statement pins the split (and its wait) ahead of the batch's DMA statements
    asm volatile("" : "+v"(ah[0]), "+v"(am[0]), "+v"(al[0]), "+v"(ah[1]), "+v"(am[1]), "+v"(al[1]));
    // chunk c + 2: B into the buffer chunk c - 1 used (free since the last barrier), then A
    dma_b(c + 2, (c + 2) % 3);
    load_a(c + 2, ra);
    const unsigned short* Bs = lds + (c % 3) * kNtBuf;
    auto rd_b = [&](int f, shortx8& bh, shortx8& bm, shortx8& bl) {
      const int j = 16 * f + cl;
      const int o = j * 32 + 8 * nt_slot(j, kq);
      if (DL_S3_DIAG == 4) {
        bh = am[0]; bm = al[1]; bl = ah[1];
      } else {
        bh = *reinterpret_cast<const shortx8*>(&Bs[o]);
        bm = *reinterpret_cast<const shortx8*>(&Bs[kNtPlane + o]);
        bl = *reinterpret_cast<const shortx8*>(&Bs[2 * kNtPlane + o]);
      }
    };
    // every fragment, also those past N (clamped weight rows, products discarded by the
    // epilogue): no per-fragment branch, so the scheduler hoists fragment f + PF's reads over
    // fragment f's MFMAs instead of each fragment waiting out its own LDS latency
    constexpr int PF = DL_S3_PF;
    shortx8 bb[PF + 1][3];
    // the fragments' LDS byte address: fragment f's rows 16f + cl sit 1,024 B apart (the
    // swizzle slot depends only on cl and kq), planes 13,312 B apart
    const uint32_t b_addr = lds_base + 2u * (uint32_t)((c % 3) * kNtBuf + cl * 32 + 8 * nt_slot(cl, kq));
#pragma unroll
    for (int i = 0; i < PF; ++i) {
      if (DL_S3_ASMB) nt_rd3(b_addr + 1024u * i, bb[i][0], bb[i][1], bb[i][2]);
      else rd_b(i, bb[i][0], bb[i][1], bb[i][2]);
    }
#pragma unroll
    for (int f = 0; f < kNtNF; ++f) {
      {
        constexpr int NB = PF + 1;
        if (f + PF < kNtNF) {
          if (DL_S3_ASMB) nt_rd3(b_addr + 1024u * (f + PF), bb[(f + PF) % NB][0], bb[(f + PF) % NB][1], bb[(f + PF) % NB][2]);
          else rd_b(f + PF, bb[(f + PF) % NB][0], bb[(f + PF) % NB][1], bb[(f + PF) % NB][2]);
        }
        if (DL_S3_ASMB) {
          shortx8 &h = bb[f % NB][0], &m = bb[f % NB][1], &l = bb[f % NB][2];
          if (f + PF < kNtNF) {           // fragments f + 1 .. f + PF may stay in flight
            if (PF == 1) DL_LDS_WAIT(3, h, m, l);
            else if (PF == 2) DL_LDS_WAIT(6, h, m, l);
            else DL_LDS_WAIT(9, h, m, l);
          } else if (f + 1 < kNtNF) {     // the tail: only fragment f + 1's reads remain younger
            DL_LDS_WAIT(3, h, m, l);
          } else {
            DL_LDS_WAIT(0, h, m, l);
          }
        }
        const shortx8 bh = bb[f % NB][0], bm = bb[f % NB][1], bl = bb[f % NB][2];
        if (DL_S3_BPF) __builtin_amdgcn_sched_barrier(0);   // keep them there
        if (DL_S3_DIAG == 2) {
          acc[0][f][0] += (float)(bh[0] ^ ah[0][1] ^ bm[2] ^ bl[3] ^ am[0][0] ^ al[0][2]);
          acc[1][f][0] += (float)(bh[1] ^ ah[1][1] ^ bm[3] ^ bl[4] ^ am[1][0] ^ al[1][2]);
        } else if (DIRECT) {
          acc[0][f] = mfma_s3_t(ah[0], am[0], al[0], bh, bm, bl, acc[0][f]);
          acc[1][f] = mfma_s3_t(ah[1], am[1], al[1], bh, bm, bl, acc[1][f]);
        } else {
          acc[0][f] = mfma_s3(ah[0], am[0], al[0], bh, bm, bl, acc[0][f]);
          acc[1][f] = mfma_s3(ah[1], am[1], al[1], bh, bm, bl, acc[1][f]);
        }
        if (DL_S3_SGB) {
          if (f + PF < kNtNF) __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);   // 3 DS reads
          __builtin_amdgcn_sched_group_barrier(0x008, 12, 0);                     // then 12 MFMAs
        }
      }
    }
    if (DL_S3_DIAG != 5) publish(c);
  };
  // pairs of unconditional steps (an odd last chunk after the loop): at the loop head the
  // latest batch is always raB's, so hipcc's own wait for raA leaves that batch in flight
  int c = 0;
  for (; c + 1 < KC; c += 2) {
    step(c, raA);
    step(c + 1, raB);
  }
  if (DL_S3_MWLATE) load_mw();
  if (c < KC) step(c, raA);
  }

  if (DL_S3_DIAG && DL_S3_DIAG != 6 && DL_S3_DIAG != 7) {   // keep the loop's results live without storing them
    float tt = 0.f;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int f = 0; f < kNtNF; ++f) tt += acc[a][f][0] + acc[a][f][3];
    if (tt == 12345.f) p.C[0] = tt;
    return;
  }
  if constexpr (DIRECT) {
    // lane (kq, cl): acc[a][f][j] = C[r0 + 16a + cl][j0 + 16f + 4kq + j].  Stores go through a
    // buffer descriptor: a piece past M or N gets an offset past its range and is dropped.
    const auto c_rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)p.C, (short)0, p.M * p.ldc * 4, 0x00020000);
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      const int row = r0 + 16 * a + cl;
#pragma unroll
      for (int f = 0; f < kNtNF; ++f) {
        const int col = j0 + 16 * f + 4 * kq;
        floatx4 v = acc[a][f];
        if (EPI == S3_RELU) {
          v[0] = fmaxf(v[0], 0.f); v[1] = fmaxf(v[1], 0.f); v[2] = fmaxf(v[2], 0.f); v[3] = fmaxf(v[3], 0.f);
        }
        if constexpr (EPI == S3_MASKBITS) {   // halfword (j0 >> 4) + f of the row, bits 4kq .. 4kq + 3
          const int hi = (j0 >> 4) + f - 2 * (j0 >> 5);
          const uint32_t m = (mw[a][hi >> 1] >> (16 * (hi & 1) + 4 * kq)) & 0xFu;
          v[0] = (m & 1u) ? v[0] : 0.f; v[1] = (m & 2u) ? v[1] : 0.f;
          v[2] = (m & 4u) ? v[2] : 0.f; v[3] = (m & 8u) ? v[3] : 0.f;
        }
        const bool ok = row < p.M && col + 4 <= p.N;
        const uint32_t off = ok ? 4u * (uint32_t)(row * p.ldc + col) : 0x80000000u;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(s3_u32x4_t, v), c_rsrc, (int)off, 0, 0);
        if (EPI == S3_RELU && p.bits) {   // the sign bitmask: row's 16 bits of fragment f from 4 lanes
          uint32_t hw = (uint32_t)((acc[a][f][0] > 0.f) | ((acc[a][f][1] > 0.f) << 1) | ((acc[a][f][2] > 0.f) << 2) |
                                   ((acc[a][f][3] > 0.f) << 3)) << (4 * kq);
          hw |= (uint32_t)__shfl_xor((int)hw, 16, 64);
          hw |= (uint32_t)__shfl_xor((int)hw, 32, 64);
          const int h = (j0 >> 4) + f;
          if (kq == 0 && row < p.M && 16 * h < p.N) p.bits[(long long)row * p.ldbits + h] = (uint16_t)hw;
        }
      }
    }
    return;
  }
  // Epilogue through LDS (the ring is free after the last barrier): per wave and per half
  // (rows 16h .. 16h+15 of its 32), the 16 x 208 tile is written from the MFMA layout, then
  // each lane moves whole 16-B row pieces: ReLU / mask reads and stores as full row segments.
  float* tile = reinterpret_cast<float*>(lds) + wid * 16 * kNtEP;
  const float* __restrict__ Mk = p.mask;
  constexpr int VPR = kNtBN / 4;                    // 52 float4 pieces per row
  constexpr int NIT = (16 * VPR + 63) / 64;         // pieces per lane per half
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    uint32_t mb[EPI == S3_MASKBITS ? NIT : 1];
    if (EPI == S3_MASKBITS) {
#pragma unroll
      for (int it = 0; it < NIT; ++it) {
        const int q = lane + 64 * it;
        const int rl = q / VPR, pc = q % VPR;
        const int row = min(r0 + 16 * h + rl, p.M - 1), col = min(j0 + 4 * pc, p.N - 1);
        mb[it] = (uint32_t)p.bits[(long long)row * p.ldbits + (col >> 4)] >> (col & 15);
      }
    }
    // the ReluGrad mask's pieces for this half are loaded first (all in flight together,
    // under the tile's LDS writes), not one dependent round trip per piece
    float4 mk4[EPI == S3_MASK ? NIT : 1];
    if (EPI == S3_MASK) {
#pragma unroll
      for (int it = 0; it < NIT; ++it) {
        const int q = lane + 64 * it;
        const int rl = q / VPR, pc = q % VPR;
        const int row = min(r0 + 16 * h + rl, p.M - 1), col = max(0, min(j0 + 4 * pc, p.N - 4));
        mk4[it] = *reinterpret_cast<const float4*>(Mk + (long long)row * p.ldm + (col & ~3));
      }
    }
#pragma unroll
    for (int f = 0; f < kNtNF; ++f)
#pragma unroll
      for (int j = 0; j < 4; ++j) tile[(4 * kq + j) * kNtEP + 16 * f + cl] = acc[h][f][j];
    __builtin_amdgcn_s_waitcnt(0xc07f);             // lgkmcnt(0): this wave's tile writes landed
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int q = lane + 64 * it;
      const int rl = q / VPR, pc = q % VPR;
      const int row = r0 + 16 * h + rl, col = j0 + 4 * pc;
      if (q >= 16 * VPR || row >= p.M || col >= p.N) continue;
      float4 v = *reinterpret_cast<const float4*>(tile + rl * kNtEP + 4 * pc);
      if (EPI == S3_RELU) {
        v.x = fmaxf(v.x, 0.f); v.y = fmaxf(v.y, 0.f); v.z = fmaxf(v.z, 0.f); v.w = fmaxf(v.w, 0.f);
      }
      if (EPI == S3_MASKBITS) {   // col % 4 == 0: the piece's four bits sit in one halfword
        const uint32_t m = mb[EPI == S3_MASKBITS ? it : 0];
        v.x = (m & 1u) ? v.x : 0.f; v.y = (m & 2u) ? v.y : 0.f; v.z = (m & 4u) ? v.z : 0.f; v.w = (m & 8u) ? v.w : 0.f;
      }
      float* dst = p.C + (long long)row * p.ldc + col;
      const float* mk = Mk + (long long)row * p.ldm + col;
      if (col + 4 <= p.N && ((reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(mk)) & 15) == 0) {
        if (EPI == S3_MASK) {
          const float4 m4 = mk4[EPI == S3_MASK ? it : 0];
          v.x = m4.x > 0.f ? v.x : 0.f; v.y = m4.y > 0.f ? v.y : 0.f;
          v.z = m4.z > 0.f ? v.z : 0.f; v.w = m4.w > 0.f ? v.w : 0.f;
        }
        *reinterpret_cast<float4*>(dst) = v;
      } else {
        const float e4[4] = {v.x, v.y, v.z, v.w};
        for (int e = 0; e < 4 && col + e < p.N; ++e) {
          float x = e4[e];
          if (EPI == S3_MASK) x = mk[e] > 0.f ? x : 0.f;
          dst[e] = x;
        }
      }
    }
    // the forward's sign bitmask, straight from the accumulators (after the half's stores are
    // issued, so the ballots run while they drain): ballot j of fragment f holds
    // rows 4kq + j (kq = bit / 16) x columns 16f + (bit % 16); lane r < 16 stores row r's halfword
    if (EPI == S3_RELU && p.bits) {
#pragma unroll
      for (int f = 0; f < kNtNF; ++f) {
        const uint64_t b0 = __ballot(acc[h][f][0] > 0.f), b1 = __ballot(acc[h][f][1] > 0.f);
        const uint64_t b2 = __ballot(acc[h][f][2] > 0.f), b3 = __ballot(acc[h][f][3] > 0.f);
        const int hw = (j0 >> 4) + f, row = r0 + 16 * h + lane;
        if (lane < 16 && row < p.M && 16 * hw < p.N) {
          const int jj = lane & 3;
          const uint64_t b = jj == 0 ? b0 : jj == 1 ? b1 : jj == 2 ? b2 : b3;
          p.bits[(long long)row * p.ldbits + hw] = (uint16_t)(b >> (16 * (lane >> 2)));
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
}

// ---------------------------------------------------------------------------- TN
// Block: 128 rows (m) x 416 columns (n) of a split-K slab, 8 waves: wave w owns rows
// 32 (w & 3) .. +32 (2 fragments) x columns 208 (w >> 2) .. +208 (13 fragments).  Per
// 32-deep batch step the f32 tiles X[k][m0..m0+128) and Y[k][0..416) are loaded into
// registers one step ahead, split, and written to LDS as three plane images each
// ([k][m], [k][n]; pitches 144 and 432 bf16 = 8 x odd words: conflict-free transposed
// reads).  Lane group kq reads batch rows 4kq..4kq+3 and 16+4kq..16+4kq+3 for both operands
// (the same k set, so the sum is unchanged).
constexpr int kTnBM = 128, kTnBN = 416, kTnKS = 32, kTnPA = 144, kTnPB = 432;
constexpr int kTnAE = kTnKS * kTnPA, kTnBE = kTnKS * kTnPB;          // elements per plane image
constexpr int kTnQA = kTnKS * kTnBM / 4, kTnQB = kTnKS * kTnBN / 4;  // float4 pieces per step
constexpr int kTnQ = (kTnQA + kTnQB + 511) / 512;
constexpr size_t kTnLds = 3 * (kTnAE + kTnBE) * sizeof(unsigned short);
static_assert(kTnQA == 2 * 512 && kTnQB == 6 * 512 + 256 && kTnQ == 9, "the TN piece mapping below");

__device__ __forceinline__ uint2 s3_lds_tr16(const unsigned short* ptr_) {
  auto lp = (__attribute__((address_space(3))) unsigned short*)(const_cast<unsigned short*>(ptr_));
  const s3_fp16x4_t v =
      __builtin_amdgcn_ds_read_tr16_b64_v4f16(reinterpret_cast<__attribute__((address_space(3))) s3_fp16x4_t*>(lp));
  return __builtin_bit_cast(uint2, v);
}

__device__ __forceinline__ shortx8 s3_tr_frag(const unsigned short* img, int pitch, int ra, int rb, int col) {
  const uint2 lo = s3_lds_tr16(&img[ra * pitch + col]);
  const uint2 hi = s3_lds_tr16(&img[rb * pitch + col]);
  return __builtin_bit_cast(shortx8, make_uint4(lo.x, lo.y, hi.x, hi.y));
}

__global__ __launch_bounds__(512) void gemm_s3_tn_kernel(S3Params p) {
  extern __shared__ __attribute__((aligned(16))) unsigned short lds[];   // [3][KS][PA] then [3][KS][PB]
  unsigned short* As = lds;
  unsigned short* Bs = lds + 3 * kTnAE;
  const float* __restrict__ X = p.A;
  const float* __restrict__ Y = reinterpret_cast<const float*>(p.B);
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int mtiles = (p.M + kTnBM - 1) / kTnBM;
  const int t = s3_xcd_tile(blockIdx.x, gridDim.x);
  const int m0 = (t % mtiles) * kTnBM, z = t / mtiles;
  const int kbeg = z * p.k_per_split;
  const int kend = min(p.K, kbeg + p.k_per_split);
  const int nk = (kend - kbeg + kTnKS - 1) / kTnKS;
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  // Pieces of a step: 1024 A pieces (32 rows x 32 float4 of X) are u = 0, 1; then 3328 B pieces
  // (32 rows x 104 float4 of Y) are u = 2..8 (u = 8: threads < 256 only).  Each thread's pieces
  // sit at fixed offsets: loads go unconditionally to clamped addresses and out-of-range
  // pieces are zeroed afterwards (no exec-masked loads).
  float4 rs[kTnQ];
  const int qa_r0 = tid >> 5, qa_c = 4 * (tid & 31);                 // u = 0: row qa_r0, u = 1: row qa_r0 + 16
  const bool qa_ok = m0 + qa_c < p.M;
  const float* xa = X + min(m0 + qa_c, p.M - 4);
  int qb_r[7], qb_c[7];
  bool qb_ok[7];
#pragma unroll
  for (int u = 0; u < 7; ++u) {
    const int qq = tid + 512 * u;
    qb_r[u] = qq / 104;
    qb_c[u] = 4 * (qq % 104);
    qb_ok[u] = qb_c[u] < p.N && (u < 6 || tid < 256);
  }
  auto load = [&](int k0) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int gk = k0 + qa_r0 + 16 * u;
      const float4 v = *reinterpret_cast<const float4*>(xa + (long long)min(gk, kend - 1) * p.lda);
      rs[u] = (qa_ok && gk < kend) ? v : z4;
    }
#pragma unroll
    for (int u = 0; u < 7; ++u) {
      const int gk = k0 + min(qb_r[u], kTnKS - 1);
      const float4 v = *reinterpret_cast<const float4*>(Y + (long long)min(gk, kend - 1) * p.ldb +
                                                          min(qb_c[u], p.N - 4));
      rs[2 + u] = (qb_ok[u] && gk < kend) ? v : z4;
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int u = 0; u < kTnQ; ++u) {
      uint32_t h0, m0_, l0, h1, m1_, l1;
      split2(rs[u].x, rs[u].y, h0, m0_, l0);
      split2(rs[u].z, rs[u].w, h1, m1_, l1);
      if (u < 2) {
        const int o = (qa_r0 + 16 * u) * kTnPA + qa_c;
        *reinterpret_cast<uint2*>(&As[o]) = make_uint2(h0, h1);
        *reinterpret_cast<uint2*>(&As[kTnAE + o]) = make_uint2(m0_, m1_);
        *reinterpret_cast<uint2*>(&As[2 * kTnAE + o]) = make_uint2(l0, l1);
      } else if (u < 8 || tid < 256) {
        const int o = qb_r[u - 2] * kTnPB + qb_c[u - 2];
        *reinterpret_cast<uint2*>(&Bs[o]) = make_uint2(h0, h1);
        *reinterpret_cast<uint2*>(&Bs[kTnBE + o]) = make_uint2(m0_, m1_);
        *reinterpret_cast<uint2*>(&Bs[2 * kTnBE + o]) = make_uint2(l0, l1);
      }
    }
  };
  floatx4 acc[2][13];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 13; ++b) acc[a][b] = floatx4{0.f, 0.f, 0.f, 0.f};
  const int wm = wid & 3, wn = wid >> 2;
  const int cl = lane & 15, kq = lane >> 4, rq = cl >> 2, cp = cl & 3;
  const int ra = 4 * kq + rq, rb = 16 + 4 * kq + rq;
  // fragments whose rows / columns lie past M / N are skipped (wave-uniform)
  const int ma_live = min(2, max(0, (p.M - (m0 + 32 * wm) + 15) / 16));
  const int nb_live = min(13, max(0, (p.N - 208 * wn + 15) / 16));
  if (nk > 0) {
    load(kbeg);
    store();
    __syncthreads();
  }
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) load(kbeg + (kt + 1) * kTnKS);
    shortx8 ah[2], am[2], al[2];
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      const int col = 32 * wm + 16 * a + 4 * cp;
      ah[a] = s3_tr_frag(As, kTnPA, ra, rb, col);
      am[a] = s3_tr_frag(As + kTnAE, kTnPA, ra, rb, col);
      al[a] = s3_tr_frag(As + 2 * kTnAE, kTnPA, ra, rb, col);
    }
#pragma unroll
    for (int b = 0; b < 13; ++b) {
      if (b < nb_live) {
        const int col = 208 * wn + 16 * b + 4 * cp;
        const shortx8 bh = s3_tr_frag(Bs, kTnPB, ra, rb, col);
        const shortx8 bm = s3_tr_frag(Bs + kTnBE, kTnPB, ra, rb, col);
        const shortx8 bl = s3_tr_frag(Bs + 2 * kTnBE, kTnPB, ra, rb, col);
#pragma unroll
        for (int a = 0; a < 2; ++a)
          if (a < ma_live) acc[a][b] = mfma_s3(ah[a], am[a], al[a], bh, bm, bl, acc[a][b]);
      }
    }
    __syncthreads();
    if (kt + 1 < nk) {
      store();
      __syncthreads();
    }
  }
  float* __restrict__ C = p.C + (long long)z * p.c_split_stride;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 13; ++b) {
      const int col = 208 * wn + 16 * b + cl;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = m0 + 32 * wm + 16 * a + 4 * kq + j;
        if (row < p.M && col < p.N) C[(long long)row * p.ldc + col] = acc[a][b][j];
      }
    }
}

// ---------------------------------------------------------------------------- TN, double-buffered
// The weight gradients again, with two LDS buffers so a step's MFMAs never wait for the next
// step's staging: per 32-deep batch step a wave computes from buffer kt & 1 while the next
// step's tiles (loaded into registers at the step's start) are split and written into the
// other buffer, and one barrier per step publishes them.  Two 73.7 KB buffers fit the 160 KB
// LDS at a 128 x 224 block (8 waves: rows 32 (w & 3) .. +32 = 2 fragments, columns 112 (w >> 2)
// .. +112 = 7 fragments); N takes ceil(N / 224) column tiles (N = 400: 2).  Pitches 144 and
// 240 bf16 (8 x odd words: conflict-free transposed reads, as above).  Out-of-range pieces
// are loaded through buffer descriptors with an offset past the range: zeros, no fixup.
constexpr int kT2BM = 128, kT2BN = 224, kT2KS = 32, kT2PA = 144, kT2PB = 240, kT2NF = 7;
constexpr int kT2AE = kT2KS * kT2PA, kT2BE = kT2KS * kT2PB;           // bf16 elements per plane image
constexpr int kT2Buf = 3 * (kT2AE + kT2BE);                           // one buffer: A planes, B planes
constexpr size_t kT2Lds = 2 * kT2Buf * sizeof(unsigned short);       // 147,456 B
constexpr int kT2QA = kT2KS * kT2BM / 4, kT2QB = kT2KS * kT2BN / 4;   // float4 pieces per step
constexpr int kT2Q = (kT2QA + kT2QB + 511) / 512;
static_assert(kT2QA == 2 * 512 && kT2QB == 3 * 512 + 256 && kT2Q == 6, "the piece mapping below");

__global__ __launch_bounds__(512) void gemm_s3_tn2_kernel(S3Params p) {
  extern __shared__ __attribute__((aligned(16))) unsigned short lds[];   // [2][3 A planes | 3 B planes]
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int mtiles = (p.M + kT2BM - 1) / kT2BM, ntiles = (p.N + kT2BN - 1) / kT2BN;
  const int t = s3_xcd_tile(blockIdx.x, gridDim.x);   // the column tiles of one (m, slab) adjacent: X shared in L2
  const int n0 = (t % ntiles) * kT2BN, m0 = ((t / ntiles) % mtiles) * kT2BM, z = t / (ntiles * mtiles);
  const int kbeg = z * p.k_per_split;
  const int kend = min(p.K, kbeg + p.k_per_split);
  const int nk = (kend - kbeg + kT2KS - 1) / kT2KS;
  const auto xr = __builtin_amdgcn_make_buffer_rsrc((void*)p.A, (short)0, p.K * p.lda * 4, 0x00020000);
  const auto yr = __builtin_amdgcn_make_buffer_rsrc((void*)p.B, (short)0, p.K * p.ldb * 4, 0x00020000);
  // this thread's pieces: u = 0, 1 -> X rows (tid >> 5) + 16u, columns 4 (tid & 31); u = 2..5 ->
  // Y piece tid + 512 (u - 2) = row / 56, column 4 (piece % 56) (u = 5: threads < 256 only)
  int pr[kT2Q], pc[kT2Q];
  bool pok[kT2Q];
#pragma unroll
  for (int u = 0; u < kT2Q; ++u) {
    if (u < 2) {
      pr[u] = (tid >> 5) + 16 * u;
      pc[u] = 4 * (tid & 31);
      pok[u] = m0 + pc[u] < p.M;
    } else {
      const int qb = tid + 512 * (u - 2);
      pr[u] = qb / (kT2BN / 4);
      pc[u] = 4 * (qb % (kT2BN / 4));
      pok[u] = n0 + pc[u] < p.N && (u < 5 || tid < 256);
    }
  }
  float4 rs[kT2Q];
  auto load = [&](int k0) {
#pragma unroll
    for (int u = 0; u < kT2Q; ++u) {
      const int gk = k0 + pr[u];
      const bool ok = pok[u] & (gk < kend);   // no short circuit: a select, not a branch
      if (u < 2) {
        const uint32_t o = 4u * (uint32_t)(gk * p.lda + m0 + pc[u]);
        rs[u] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(xr, (int)(ok ? o : 0x80000000u), 0, 0));
      } else {
        const uint32_t o = 4u * (uint32_t)(gk * p.ldb + n0 + pc[u]);
        rs[u] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(yr, (int)(ok ? o : 0x80000000u), 0, 0));
      }
    }
  };
  auto store = [&](int buf) {
    unsigned short* As = lds + buf * kT2Buf;
    unsigned short* Bs = As + 3 * kT2AE;
#pragma unroll
    for (int u = 0; u < kT2Q; ++u) {
      if (u == 5 && tid >= 256) continue;
      uint32_t h0, m0_, l0, h1, m1_, l1;
      if (DL_S3_DIAG == 6) {   // timing only: no split
        h0 = __float_as_uint(rs[u].x); m0_ = __float_as_uint(rs[u].y); l0 = h0;
        h1 = __float_as_uint(rs[u].z); m1_ = __float_as_uint(rs[u].w); l1 = h1;
      } else {
        split2(rs[u].x, rs[u].y, h0, m0_, l0);
        split2(rs[u].z, rs[u].w, h1, m1_, l1);
      }
      unsigned short* img = u < 2 ? As : Bs;
      const int pe = u < 2 ? kT2AE : kT2BE;
      const int o = pr[u] * (u < 2 ? kT2PA : kT2PB) + pc[u];
      *reinterpret_cast<uint2*>(&img[o]) = make_uint2(h0, h1);
      *reinterpret_cast<uint2*>(&img[pe + o]) = make_uint2(m0_, m1_);
      *reinterpret_cast<uint2*>(&img[2 * pe + o]) = make_uint2(l0, l1);
    }
  };
  floatx4 acc[2][kT2NF];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < kT2NF; ++b) acc[a][b] = floatx4{0.f, 0.f, 0.f, 0.f};
  const int wm = wid & 3, wn = wid >> 2;
  const int cl = lane & 15, kq = lane >> 4, rq = cl >> 2, cp = cl & 3;
  const int ra = 4 * kq + rq, rb = 16 + 4 * kq + rq;
  auto compute = [&](int buf) {   // every fragment (zeros past M / N): no branches between them
    const unsigned short* As = lds + buf * kT2Buf;
    const unsigned short* Bs = As + 3 * kT2AE;
    shortx8 ah[2], am[2], al[2];
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      const int col = 32 * wm + 16 * a + 4 * cp;
      ah[a] = s3_tr_frag(As, kT2PA, ra, rb, col);
      am[a] = s3_tr_frag(As + kT2AE, kT2PA, ra, rb, col);
      al[a] = s3_tr_frag(As + 2 * kT2AE, kT2PA, ra, rb, col);
    }
#pragma unroll
    for (int b = 0; b < kT2NF; ++b) {
      const int col = 112 * wn + 16 * b + 4 * cp;
      const shortx8 bh = s3_tr_frag(Bs, kT2PB, ra, rb, col);
      const shortx8 bm = s3_tr_frag(Bs + kT2BE, kT2PB, ra, rb, col);
      const shortx8 bl = s3_tr_frag(Bs + 2 * kT2BE, kT2PB, ra, rb, col);
#pragma unroll
      for (int a = 0; a < 2; ++a) acc[a][b] = mfma_s3(ah[a], am[a], al[a], bh, bm, bl, acc[a][b]);
    }
  };
  if (DL_S3_TNSTAG) {
    // Staggered roles (MI355X_MICROARCH.md, two waves per SIMD: waves w and w + 4 share one):
    // waves 0-3 run [MFMAs of step kt][split + store of step kt + 1], waves 4-7 the reverse, so
    // on every SIMD one wave's VALU/LDS work runs beside the other's MFMAs.  The registers
    // hold step kt + 1's tiles from the load issued after the previous store; the barrier
    // waits only for this wave's LDS writes (a __syncthreads would also drain the loads in
    // flight, vmcnt(0)).
    if (nk > 0) {
      load(kbeg);
      store(0);
      if (nk > 1) load(kbeg + kT2KS);
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0)
    __builtin_amdgcn_s_barrier();
    const bool late = wid >= 4;
    for (int kt = 0; kt < nk; ++kt) {
      const bool more = kt + 1 < nk;
      if (!late) compute(kt & 1);
      if (more) {
        store((kt + 1) & 1);            // the other buffer: its last readers passed the previous barrier
        if (kt + 2 < nk) load(kbeg + (kt + 2) * kT2KS);
      }
      if (late) compute(kt & 1);
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_s_barrier();
    }
  } else {
    if (nk > 0) {
      load(kbeg);
      store(0);
    }
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const bool more = kt + 1 < nk;
      if (more) load(kbeg + (kt + 1) * kT2KS);
      compute(kt & 1);
      if (more) store((kt + 1) & 1);   // the other buffer: its last readers passed the previous barrier
      __syncthreads();
    }
  }
  float* __restrict__ C = p.C + (long long)z * p.c_split_stride;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < kT2NF; ++b) {
      const int col = n0 + 112 * wn + 16 * b + cl;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = m0 + 32 * wm + 16 * a + 4 * kq + j;
        if (row < p.M && col < p.N) C[(long long)row * p.ldc + col] = acc[a][b][j];
      }
    }
}

// ---------------------------------------------------------------------------- TN, interleaved
// The double-buffered TN kernel with its staging moved under the MFMAs: the f32 tiles are
// loaded two steps ahead (two register sets), and step kt + 1's six pieces per thread are split
// and written to the other LDS buffer between step kt's fragment groups (piece b after fragment
// b's twelve MFMAs), so each wave's VALU split and LDS stores issue while its MFMAs execute
// instead of in a phase of their own between barriers (tn2: MFMA busy about half the loop).
// Same tiles, images, fragment reads and k order as tn2: the same sums bit for bit.
#ifndef DL_S3_TN3
#define DL_S3_TN3 1   // weight gradients: the interleaved kernel (0: tn2)
#endif


// SKIP: a wave whose row fragments lie past M (the last row tile: M = 400 leaves 1 of its 8
// fragment rows in range, 432 leaves 3) skips their MFMAs and fragment reads, and the waves of
// one fragment row sit on different SIMDs (wm = wid >> 1), so such a block costs about its
// split work plus the valid rows' MFMAs instead of a full tile's.
template <bool SKIP>
__global__ __launch_bounds__(512) void gemm_s3_tn3_kernel(S3Params p) {
  extern __shared__ __attribute__((aligned(16))) unsigned short lds[];   // [2][3 A planes | 3 B planes]
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int mtiles = (p.M + kT2BM - 1) / kT2BM, ntiles = (p.N + kT2BN - 1) / kT2BN;
  const int t = s3_xcd_tile(blockIdx.x, gridDim.x);
  const int n0 = (t % ntiles) * kT2BN, m0 = ((t / ntiles) % mtiles) * kT2BM, z = t / (ntiles * mtiles);
  const int kbeg = z * p.k_per_split;
  const int kend = min(p.K, kbeg + p.k_per_split);
  const int nk = (kend - kbeg + kT2KS - 1) / kT2KS;
  const auto xr = __builtin_amdgcn_make_buffer_rsrc((void*)p.A, (short)0, p.K * p.lda * 4, 0x00020000);
  const auto yr = __builtin_amdgcn_make_buffer_rsrc((void*)p.B, (short)0, p.K * p.ldb * 4, 0x00020000);
  int pr[kT2Q], pc[kT2Q];
#pragma unroll
  for (int u = 0; u < kT2Q; ++u) {
    if (u < 2) {
      pr[u] = (tid >> 5) + 16 * u;
      pc[u] = 4 * (tid & 31);
    } else {
      const int qb = tid + 512 * (u - 2);
      pr[u] = qb / (kT2BN / 4);
      pc[u] = 4 * (qb % (kT2BN / 4));
    }
  }
  // Loads need no bounds selects: a piece past M / N (or one of the unused u = 5 pieces) only
  // reaches rows / columns of C the epilogue discards, whatever it reads; a split's steps end at
  // its kend (k_per_split is a multiple of the step) except the last split's, whose rows past K
  // fall past the descriptor's range and read as zeros; loads for steps past nk are never
  // stored.  So each piece's offset is a per-thread constant plus the step's (one add).
  // (the host checks (K + 1) * ld * 4 < 2^31: no offset wraps into range)
  uint32_t vo[kT2Q];
#pragma unroll
  for (int u = 0; u < kT2Q; ++u)
    vo[u] = u < 2 ? 4u * (uint32_t)(pr[u] * p.lda + m0 + pc[u]) : 4u * (uint32_t)(pr[u] * p.ldb + n0 + pc[u]);
  auto load = [&](int k0, float4 (&rs)[kT2Q]) {
    const uint32_t sa = 4u * (uint32_t)(k0 * p.lda), sb = 4u * (uint32_t)(k0 * p.ldb);
#pragma unroll
    for (int u = 0; u < kT2Q; ++u) {
      if (u < 2)
        rs[u] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(xr, (int)(vo[u] + sa), 0, 0));
      else
        rs[u] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(yr, (int)(vo[u] + sb), 0, 0));
    }
  };
  auto store_piece = [&](int buf, int u, const float4& r) {
    if (u == 5 && tid >= 256) return;
    unsigned short* As = lds + buf * kT2Buf;
    unsigned short* Bs = As + 3 * kT2AE;
    uint32_t h0, m0_, l0, h1, m1_, l1;
    if (DL_S3_DIAG == 6) {   // timing only: no split
      h0 = __float_as_uint(r.x); m0_ = __float_as_uint(r.y); l0 = h0;
      h1 = __float_as_uint(r.z); m1_ = __float_as_uint(r.w); l1 = h1;
    } else {
      split2(r.x, r.y, h0, m0_, l0);
      split2(r.z, r.w, h1, m1_, l1);
    }
    unsigned short* img = u < 2 ? As : Bs;
    const int pe = u < 2 ? kT2AE : kT2BE;
    const int o = pr[u] * (u < 2 ? kT2PA : kT2PB) + pc[u];
    *reinterpret_cast<uint2*>(&img[o]) = make_uint2(h0, h1);
    *reinterpret_cast<uint2*>(&img[pe + o]) = make_uint2(m0_, m1_);
    *reinterpret_cast<uint2*>(&img[2 * pe + o]) = make_uint2(l0, l1);
  };
  floatx4 acc[2][kT2NF];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < kT2NF; ++b) acc[a][b] = floatx4{0.f, 0.f, 0.f, 0.f};
  const int wm = SKIP ? wid >> 1 : wid & 3, wn = SKIP ? wid & 1 : wid >> 2;
  const int cl = lane & 15, kq = lane >> 4, rq = cl >> 2, cp = cl & 3;
  const int ra = 4 * kq + rq, rb = 16 + 4 * kq + rq;
  // some row of this wave's fragments inside M (wave-uniform)
  const bool live = __builtin_amdgcn_readfirstlane(m0 + 32 * wm) < p.M;
  // step kt from buffer kt & 1; `nx` (step kt + 1's tiles) split into buffer (kt + 1) & 1 piece by
  // piece between the fragment groups (skipped past the last step: nothing left to stage)
  auto step = [&](int kt, int buf, const float4 (&nx)[kT2Q]) {   // buf == kt & 1, a literal at each call
    const bool more = kt + 1 < nk;
    const unsigned short* As = lds + buf * kT2Buf;
    const unsigned short* Bs = As + 3 * kT2AE;
    shortx8 ah[2], am[2], al[2];
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      const int col = 32 * wm + 16 * a + 4 * cp;
      ah[a] = s3_tr_frag(As, kT2PA, ra, rb, col);
      am[a] = s3_tr_frag(As + kT2AE, kT2PA, ra, rb, col);
      al[a] = s3_tr_frag(As + 2 * kT2AE, kT2PA, ra, rb, col);
    }
    shortx8 bb[2][3];
    {
      const int col = 112 * wn + 4 * cp;
      bb[0][0] = s3_tr_frag(Bs, kT2PB, ra, rb, col);
      bb[0][1] = s3_tr_frag(Bs + kT2BE, kT2PB, ra, rb, col);
      bb[0][2] = s3_tr_frag(Bs + 2 * kT2BE, kT2PB, ra, rb, col);
    }
#pragma unroll
    for (int b = 0; b < kT2NF; ++b) {
      if (b + 1 < kT2NF) {   // fragment b + 1's reads ahead of fragment b's MFMAs
        const int col = 112 * wn + 16 * (b + 1) + 4 * cp;
        bb[(b + 1) & 1][0] = s3_tr_frag(Bs, kT2PB, ra, rb, col);
        bb[(b + 1) & 1][1] = s3_tr_frag(Bs + kT2BE, kT2PB, ra, rb, col);
        bb[(b + 1) & 1][2] = s3_tr_frag(Bs + 2 * kT2BE, kT2PB, ra, rb, col);
      }
#pragma unroll
      for (int a = 0; a < 2; ++a)
        acc[a][b] = mfma_s3(ah[a], am[a], al[a], bb[b & 1][0], bb[b & 1][1], bb[b & 1][2], acc[a][b]);
      if (b < kT2Q && more) store_piece(buf ^ 1, b, nx[b]);
    }
  };
  // a wave whose rows all lie past M only stages its pieces (wave-uniform branch)
  auto stage_only = [&](int kt, int buf, const float4 (&nx)[kT2Q]) {
    if (kt + 1 < nk) {
#pragma unroll
      for (int u = 0; u < kT2Q; ++u) store_piece(buf ^ 1, u, nx[u]);
    }
  };
  float4 rA[kT2Q], rB[kT2Q];
  if (nk > 0) {
    load(kbeg, rA);
    load(kbeg + kT2KS, rB);   // past kend: never stored
#pragma unroll
    for (int u = 0; u < kT2Q; ++u) store_piece(0, u, rA[u]);
  }
  __syncthreads();
  // pairs of steps: at step kt the registers of kt + 1 are stored and those of kt (already in
  // LDS) take step kt + 2's loads
  // (a bare s_barrier after lgkmcnt(0): __syncthreads' fence would also wait for the loads of
  // two steps ahead)
  int kt = 0;
  if (!SKIP || live) {
    for (; kt + 1 < nk; kt += 2) {
      load(kbeg + (kt + 2) * kT2KS, rA);
      step(kt, 0, rB);
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_s_barrier();
      load(kbeg + (kt + 3) * kT2KS, rB);
      step(kt + 1, 1, rA);
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_s_barrier();
    }
    if (kt < nk) step(kt, 0, rB);
  } else {
    for (; kt + 1 < nk; kt += 2) {
      load(kbeg + (kt + 2) * kT2KS, rA);
      stage_only(kt, 0, rB);
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_s_barrier();
      load(kbeg + (kt + 3) * kT2KS, rB);
      stage_only(kt + 1, 1, rA);
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_s_barrier();
    }
  }
  float* __restrict__ C = p.C + (long long)z * p.c_split_stride;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < kT2NF; ++b) {
      const int col = n0 + 112 * wn + 16 * b + cl;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = m0 + 32 * wm + 16 * a + 4 * kq + j;
        if (row < p.M && col < p.N) C[(long long)row * p.ldc + col] = acc[a][b][j];
      }
    }
}

// ---------------------------------------------------------------------------- split
// dst plane q (q = 0 hi, 1 mid, 2 lo) at dst + q * plane: element (r, c) of src [rows][cols]
// (ld lds) goes to [r][c] (ldd), or to [c][r] when transposed.
__global__ __launch_bounds__(256) void split3_kernel(const float* __restrict__ src, int rows, int cols, int lds,
                                                     int transpose, unsigned short* __restrict__ dst, int ldd,
                                                     long long plane) {
  const long long n = (long long)rows * cols;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const int r = (int)(i / cols), c = (int)(i % cols);
    uint32_t h, m, l;
    split2(src[(long long)r * lds + c], 0.f, h, m, l);
    // the k index (the planes' row position) in the NT kernels' order (common.h s3_kpos)
    const long long o = transpose ? (long long)c * ldd + s3_kpos(r, rows) : (long long)r * ldd + s3_kpos(c, cols);
    dst[o] = (unsigned short)h;
    dst[plane + o] = (unsigned short)m;
    dst[2 * plane + o] = (unsigned short)l;
  }
}

}  // namespace dl

using namespace dl;

extern "C" int dl_s3_kperm(void) { return DL_S3_KPERM; }

// DL_S3_DIRECT=0 in the environment: the NT epilogue through LDS (A/B measurements)
static bool s3_direct_enabled() {
  static const bool on = [] {
    const char* e = getenv("DL_S3_DIRECT");
    return !(e && e[0] == '0');
  }();
  return on;
}

// DL_S3_TNSKIP=0: every wave of a TN block runs all its MFMAs (A/B measurements)
static bool s3_tnskip_enabled() {
  static const bool on = [] {
    const char* e = getenv("DL_S3_TNSKIP");
    return !(e && e[0] == '0');
  }();
  return on;
}

extern "C" int dl_split3(const float* src, int32_t rows, int32_t cols, int32_t lds, int32_t transpose,
                         uint16_t* dst, int32_t ldd, int64_t plane_stride, void* stream) {
  DL_CHECK_ARG(src && dst, "NULL pointer");
  DL_CHECK_ARG(rows >= 0 && cols >= 0 && lds >= cols, "bad src shape");
  DL_CHECK_ARG(ldd >= (transpose ? rows : cols), "ldd too small");
  DL_CHECK_ARG(plane_stride >= (long long)ldd * (transpose ? cols : rows), "plane stride too small");
  const long long n = (long long)rows * cols;
  if (n == 0) return 0;
  long long blocks = (n + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(split3_kernel, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), src, rows, cols, lds,
                     transpose, reinterpret_cast<unsigned short*>(dst), ldd, (long long)plane_stride);
  DL_RETURN_LAUNCH("dl_split3");
}

static int s3_nt_check(int32_t M, int32_t N, int32_t K, const float* A, int32_t lda, const uint16_t* Bp,
                       int32_t ldb, int64_t b_plane, float* C, int32_t ldc, int32_t epi, const float* mask,
                       uint16_t* bits, int32_t ldbits) {
  DL_CHECK_ARG(M >= 0 && N >= 0 && K >= 0, "negative dims");
  DL_CHECK_ARG(A && Bp && C, "NULL operand");
  DL_CHECK_ARG(K % 8 == 0 && K >= 8, "K %d must be a positive multiple of 8", K);
  DL_CHECK_ARG(lda % 4 == 0 && lda >= K && ldb % 8 == 0 && ldb >= K && ldc >= N, "bad leading dims");
  DL_CHECK_ARG(((uintptr_t)A % 16) == 0 && ((uintptr_t)Bp % 16) == 0 && b_plane % 8 == 0,
               "A / B planes must be 16-byte aligned");
  DL_CHECK_ARG(b_plane >= (long long)ldb * N, "plane stride too small");
  DL_CHECK_ARG(epi >= 0 && epi <= 3, "bad epilogue %d", epi);
  DL_CHECK_ARG(epi != S3_MASK || mask, "mask epilogue needs mask");
  DL_CHECK_ARG(epi != S3_MASKBITS || bits, "bitmask epilogue needs the bitmask");
  DL_CHECK_ARG(!bits || ldbits >= (N + 15) / 16, "ldbits %d < %d halfwords", ldbits, (N + 15) / 16);
  DL_CHECK_ARG(!bits || epi == S3_RELU || epi == S3_MASKBITS, "a bitmask goes with the relu / bitmask epilogues");
  DL_CHECK_ARG((long long)M * lda * 4 < (1LL << 31), "A spans %lld bytes: past the 31-bit buffer range",
               (long long)M * lda * 4);
  return 0;
}

static bool s3_nt_direct(int32_t M, int32_t N, int32_t ldc, int32_t epi, const uint16_t* bits, int32_t ldbits) {
  return s3_direct_enabled() && N % 4 == 0 && ldc % 4 == 0 && (!bits || ldbits % 2 == 0) &&
         epi != S3_MASK && (long long)M * ldc * 4 < (1LL << 31) &&
         (epi != S3_MASKBITS || ldbits >= 2 * ((((int)ceil_div(N, kNtBN) - 1) * kNtBN >> 5) + 7));
}

extern "C" int dl_gemm_s3_nt_bits(int32_t M, int32_t N, int32_t K, const float* A, int32_t lda, const uint16_t* Bp,
                                  int32_t ldb, int64_t b_plane, float* C, int32_t ldc, int32_t epi, const float* mask,
                                  int32_t ldm, uint16_t* bits, int32_t ldbits, void* stream) {
  if (int rc = s3_nt_check(M, N, K, A, lda, Bp, ldb, b_plane, C, ldc, epi, mask, bits, ldbits)) return rc;
  if (M == 0 || N == 0) return 0;
  S3Params p{};
  p.A = A; p.B = Bp; p.C = C; p.mask = mask;
  p.M = M; p.N = N; p.K = K; p.lda = lda; p.ldb = ldb; p.ldc = ldc; p.ldm = ldm; p.b_plane = b_plane;
  p.bits = bits; p.ldbits = ldbits;
  hipStream_t s = as_stream(stream);
  const bool direct = s3_nt_direct(M, N, ldc, epi, bits, ldbits);
  const int tiles = (int)(ceil_div(M, kNtBM) * ceil_div(N, kNtBN));
  if (direct) {
    if (epi == S3_STORE) hipLaunchKernelGGL((gemm_s3_nt_kernel<S3_STORE, true>), dim3(tiles), dim3(512), kNtLds, s, p);
    else if (epi == S3_RELU) hipLaunchKernelGGL((gemm_s3_nt_kernel<S3_RELU, true>), dim3(tiles), dim3(512), kNtLds, s, p);
    else hipLaunchKernelGGL((gemm_s3_nt_kernel<S3_MASKBITS, true>), dim3(tiles), dim3(512), kNtLds, s, p);
  } else if (epi == S3_STORE) hipLaunchKernelGGL(gemm_s3_nt_kernel<S3_STORE>, dim3(tiles), dim3(512), kNtLds, s, p);
  else if (epi == S3_RELU) hipLaunchKernelGGL(gemm_s3_nt_kernel<S3_RELU>, dim3(tiles), dim3(512), kNtLds, s, p);
  else if (epi == S3_MASK) hipLaunchKernelGGL(gemm_s3_nt_kernel<S3_MASK>, dim3(tiles), dim3(512), kNtLds, s, p);
  else hipLaunchKernelGGL(gemm_s3_nt_kernel<S3_MASKBITS>, dim3(tiles), dim3(512), kNtLds, s, p);
  DL_RETURN_LAUNCH("dl_gemm_s3_nt");
}

static int s3_nt_gather_launch(int32_t M, int32_t N, int32_t K, const float* A, int32_t lda, const float* table,
                               int64_t n_rows, int32_t table_ld, const int64_t* ids, const int32_t* ids32,
                               int32_t ids_ld, int64_t id_offset, int32_t zero_row0, int32_t fields, int32_t emb_dim,
                               const uint16_t* Bp, int32_t ldb, int64_t b_plane, float* C, int32_t ldc, int32_t epi,
                               uint16_t* bits, int32_t ldbits, float* a_store, void* stream,
                               const uint32_t* gofs = nullptr) {
  if (int rc = s3_nt_check(M, N, K, A, lda, Bp, ldb, b_plane, C, ldc, epi, nullptr, bits, ldbits)) return rc;
  DL_CHECK_ARG(epi == S3_STORE || epi == S3_RELU, "gather: epilogue %d (store / relu only)", epi);
  DL_CHECK_ARG(table && (ids || ids32 || gofs), "gather: NULL table / ids");
  DL_CHECK_ARG(emb_dim == 8 || emb_dim == 16 || emb_dim == 32 || emb_dim == 64, "gather: emb_dim %d", emb_dim);
  DL_CHECK_ARG(fields > 0 && fields <= kNtGmaxF, "gather: %d fields (1..%d)", fields, kNtGmaxF);
  DL_CHECK_ARG((fields * emb_dim) % 32 == 0 && fields * emb_dim <= K,
               "gather: the gathered columns (%d) must be whole 32-deep chunks within K", fields * emb_dim);
  DL_CHECK_ARG(table_ld >= emb_dim && table_ld % 4 == 0 && (uintptr_t)table % 16 == 0,
               "gather: the table rows must be 16-B aligned");
  DL_CHECK_ARG(ids_ld >= fields && n_rows > 0, "gather: bad id matrix / rows");
  DL_CHECK_ARG((unsigned long long)n_rows * table_ld * 4 < kNtGmasked,
               "gather: the table spans %lld bytes (past the 32-bit buffer range)", (long long)n_rows * table_ld * 4);
  if (M == 0 || N == 0) return 0;
  S3Params p{};
  p.A = A; p.B = Bp; p.C = C;
  p.M = M; p.N = N; p.K = K; p.lda = lda; p.ldb = ldb; p.ldc = ldc; p.b_plane = b_plane;
  p.bits = bits; p.ldbits = ldbits;
  p.G = table; p.ids = ids; p.ids32 = ids32; p.a_store = a_store;
  p.id_off = id_offset; p.n_rows = n_rows; p.ids_ld = ids_ld; p.g_ld = table_ld;
  p.g_fields = fields; p.g_esh = __builtin_ctz(emb_dim); p.g_chunks = fields * emb_dim / 32;
  p.zero_row0 = zero_row0 ? 1 : 0;
  p.g_bytes = (unsigned)(n_rows * table_ld * 4);
  p.gofs = gofs;
  hipStream_t s = as_stream(stream);
  const bool direct = s3_nt_direct(M, N, ldc, epi, bits, ldbits);
  const int tiles = (int)(ceil_div(M, kNtBM) * ceil_div(N, kNtBN));
  const size_t lds = kNtLds + (size_t)fields * kNtGfs * 4;
#define DL_S3G(E_, D_, ST_) hipLaunchKernelGGL((gemm_s3_nt_kernel<E_, D_, true, ST_>), dim3(tiles), dim3(512), lds, s, p)
  if (a_store) {   // the training form: int32 rows, x0 written
    if (direct) { if (epi == S3_STORE) DL_S3G(S3_STORE, true, true); else DL_S3G(S3_RELU, true, true); }
    else if (epi == S3_STORE) DL_S3G(S3_STORE, false, true);
    else DL_S3G(S3_RELU, false, true);
  } else if (direct) {
    if (epi == S3_STORE) DL_S3G(S3_STORE, true, false); else DL_S3G(S3_RELU, true, false);
  } else if (epi == S3_STORE) DL_S3G(S3_STORE, false, false);
  else DL_S3G(S3_RELU, false, false);
#undef DL_S3G
  DL_RETURN_LAUNCH("dl_gemm_s3_nt_gather");
}

extern "C" int dl_gemm_s3_nt_gather(int32_t M, int32_t N, int32_t K, const float* A, int32_t lda,
                                    const float* table, int64_t n_rows, int32_t table_ld, const int64_t* ids,
                                    int32_t ids_ld, int64_t id_offset, int32_t zero_row0, int32_t fields,
                                    int32_t emb_dim, const uint16_t* Bp, int32_t ldb, int64_t b_plane, float* C,
                                    int32_t ldc, int32_t epi, uint16_t* bits, int32_t ldbits, void* stream) {
  DL_CHECK_ARG(ids, "gather: NULL ids");
  return s3_nt_gather_launch(M, N, K, A, lda, table, n_rows, table_ld, ids, nullptr, ids_ld, id_offset, zero_row0,
                             fields, emb_dim, Bp, ldb, b_plane, C, ldc, epi, bits, ldbits, nullptr, stream);
}

extern "C" int dl_gemm_s3_nt_gather_rows(int32_t M, int32_t N, int32_t K, float* A, int32_t lda, const float* rows,
                                         int64_t n_rows, int32_t rows_ld, const int32_t* idx, int32_t idx_ld,
                                         int32_t idx_base, int32_t fields, int32_t emb_dim, const uint16_t* Bp,
                                         int32_t ldb, int64_t b_plane, float* C, int32_t ldc, int32_t epi,
                                         uint16_t* bits, int32_t ldbits, void* stream) {
  DL_CHECK_ARG(idx && A, "gather rows: NULL idx / A");
  DL_CHECK_ARG(idx_base >= 0, "gather rows: idx_base %d", idx_base);
  return s3_nt_gather_launch(M, N, K, A, lda, rows, n_rows, rows_ld, nullptr, idx, idx_ld, idx_base, 0, fields,
                             emb_dim, Bp, ldb, b_plane, C, ldc, epi, bits, ldbits, A, stream);
}

extern "C" int dl_gemm_s3_nt_gather_tab(int32_t M, int32_t N, int32_t K, const float* A, int32_t lda,
                                        const float* table, int64_t n_rows, int32_t table_ld, const uint32_t* gtab,
                                        int32_t fields, int32_t emb_dim, const uint16_t* Bp, int32_t ldb,
                                        int64_t b_plane, float* C, int32_t ldc, int32_t epi, uint16_t* bits,
                                        int32_t ldbits, void* stream) {
  DL_CHECK_ARG(gtab, "gather tab: NULL offset table");
  DL_CHECK_ARG(((uintptr_t)gtab % 16) == 0, "gather tab: the offset table must be 16-B aligned");
  return s3_nt_gather_launch(M, N, K, A, lda, table, n_rows, table_ld, nullptr, nullptr, fields, 0, 0, fields, emb_dim,
                             Bp, ldb, b_plane, C, ldc, epi, bits, ldbits, nullptr, stream, gtab);
}

extern "C" int dl_gemm_s3_nt(int32_t M, int32_t N, int32_t K, const float* A, int32_t lda, const uint16_t* Bp,
                             int32_t ldb, int64_t b_plane, float* C, int32_t ldc, int32_t epi, const float* mask,
                             int32_t ldm, void* stream) {
  DL_CHECK_ARG(epi >= 0 && epi <= 2, "bad epilogue %d", epi);
  return dl_gemm_s3_nt_bits(M, N, K, A, lda, Bp, ldb, b_plane, C, ldc, epi, mask, ldm, nullptr, 0, stream);
}

extern "C" int dl_gemm_s3_tn(int32_t M, int32_t N, int32_t K, const float* X, int32_t lda, const float* Y,
                             int32_t ldb, float* C, int32_t ldc, int32_t splits, int64_t c_split_stride,
                             void* stream) {
  DL_CHECK_ARG(M >= 0 && N >= 0 && K >= 0, "negative dims");
  DL_CHECK_ARG(X && Y && C, "NULL operand");
  DL_CHECK_ARG(DL_S3_TN2 || N <= kTnBN, "N %d > %d", N, kTnBN);
  DL_CHECK_ARG(M % 4 == 0 && N % 4 == 0 && (M == 0 || M >= 4) && (N == 0 || N >= 4), "M, N must be multiples of 4");
  DL_CHECK_ARG(!DL_S3_TN2 || ((long long)(K + 1) * lda * 4 < (1LL << 31) && (long long)(K + 1) * ldb * 4 < (1LL << 31)),
               "X / Y past the 31-bit buffer range");
  DL_CHECK_ARG(lda % 4 == 0 && ldb % 4 == 0 && lda >= (M + 3) / 4 * 4 && ldb >= (N + 3) / 4 * 4 && ldc >= N,
               "bad leading dims");
  DL_CHECK_ARG(((uintptr_t)X % 16) == 0 && ((uintptr_t)Y % 16) == 0, "X / Y must be 16-byte aligned");
  if (splits < 1) splits = 1;
  DL_CHECK_ARG(splits == 1 || c_split_stride >= (long long)ldc * M, "slab stride too small");
  if (M == 0 || N == 0) return 0;
  S3Params p{};
  p.A = X; p.B = Y; p.C = C;
  p.M = M; p.N = N; p.K = K; p.lda = lda; p.ldb = ldb; p.ldc = ldc;
  int kps = (int)ceil_div(K > 0 ? K : 1, splits);
  kps = (kps + 63) / 64 * 64;                    // callers sum ceil(K / kps) slabs at this rounding
  p.k_per_split = kps;
  p.c_split_stride = c_split_stride;
  splits = (int)ceil_div(K > 0 ? K : 1, kps);
  if (DL_S3_TN2 && DL_S3_TN3) {
    const int tiles = (int)(ceil_div(M, kT2BM) * ceil_div(N, kT2BN));
    if (s3_tnskip_enabled())
      hipLaunchKernelGGL(gemm_s3_tn3_kernel<true>, dim3((unsigned)(tiles * splits)), dim3(512), kT2Lds, as_stream(stream), p);
    else
      hipLaunchKernelGGL(gemm_s3_tn3_kernel<false>, dim3((unsigned)(tiles * splits)), dim3(512), kT2Lds, as_stream(stream), p);
  } else if (DL_S3_TN2) {
    const int tiles = (int)(ceil_div(M, kT2BM) * ceil_div(N, kT2BN));
    hipLaunchKernelGGL(gemm_s3_tn2_kernel, dim3((unsigned)(tiles * splits)), dim3(512), kT2Lds, as_stream(stream), p);
  } else {
    const int mtiles = (int)ceil_div(M, kTnBM);
    hipLaunchKernelGGL(gemm_s3_tn_kernel, dim3((unsigned)(mtiles * splits)), dim3(512), kTnLds, as_stream(stream), p);
  }
  DL_RETURN_LAUNCH("dl_gemm_s3_tn");
}
