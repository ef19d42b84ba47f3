// Hand-written stable LSD radix sort of (key, value) pairs (rsort.hip), used by the batch
// index build (index.hip: dl_index_build, dl_sort_unique).  No library kernels, no host
// synchronisation, no allocation: every size it needs after the first pass (the number of
// valid keys) stays on the device, so a whole index build can be captured in a hipGraph.
#pragma once
#include "common.h"

namespace dl {

// Where the first pass reads its (key, value) pairs from.
struct RsSource {
  // kind 0: keys[e], value e; a key of 0xFFFFFFFF (-1) is dropped          (dl_sort_unique)
  // kind 1: the batch's table references, value e = sample * slots + slot (dl_index_build):
  //         key (owner << 27) | local of the referenced row, or no key (row 0 under the
  //         zero-row rule); out-of-range ids set *err and give no key; inv[e] = -1 for
  //         every reference without a key
  int kind;
  const uint32_t* keys;
  dl_emb_layout L;
  const int64_t* cate;
  int world, rep_below;
  int32_t* err;
  int32_t* inv;
  // kind 1 with n1 > 0 (dl_index_build_pair): references e >= n1 are a second id set — the
  // references of (L2, cate2) numbered from n1, keyed (1 << 27) | row in owner group 1 (the
  // first set keeps owner 0: world must be 1)
  long long n1;
  dl_emb_layout L2;
  const int64_t* cate2;
};

// Bytes of workspace rsort_pairs needs for n pairs (16-B aligned pieces).
size_t rsort_workspace_bytes(int64_t n);

// Sorts the source's valid pairs by key (stable: equal keys keep ascending value order) into
// out_keys / out_vals[0 .. *n_valid).  Keys are ordered by their compressed form
// (key >> 27) * lrange + (key & (2^27 - 1)) when lrange > 0 (owner-major index keys), by the
// key itself when lrange == 0; `bits` = significant bits of the compressed key.
int rsort_pairs(const RsSource& src, int64_t n, uint32_t lrange, int bits, void* ws, size_t ws_bytes,
                uint32_t* out_keys, int32_t* out_vals, int32_t* n_valid, hipStream_t s);

}  // namespace dl
