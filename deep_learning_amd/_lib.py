"""ctypes binding of the HIP C ABI (include/dlamd.h) — the only way the package
reaches the GPU kernels.  There is no CPU fallback: if the in-tree
``libdlamd.so`` is missing or a call fails, an exception is raised.
"""
import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libdlamd%s.so" % ("_" + os.environ["DLAMD_VARIANT"]
                                                   if os.environ.get("DLAMD_VARIANT") else ""))


class DLError(RuntimeError):
    pass


class EmbLayout(C.Structure):
    """Mirror of ``dl_emb_layout`` (include/dlamd.h)."""
    _fields_ = [
        ("n_rows", C.c_int64), ("fm_cont_offset", C.c_int64), ("fm_cate_offset", C.c_int64),
        ("deep_cate_offset", C.c_int64),
        ("batch", C.c_int32), ("emb_dim", C.c_int32), ("cont_fields", C.c_int32),
        ("vector_size", C.c_int32), ("cate_fields", C.c_int32), ("cate_ld", C.c_int32),
        ("fm_cont", C.c_int32), ("use_fm", C.c_int32), ("fm_extra", C.c_int32),
        ("zero_row0", C.c_int32), ("x0_ld", C.c_int32), ("x0_cont_col", C.c_int32),
        ("x0_vec_col", C.c_int32), ("x0_cat_col", C.c_int32), ("x0_pool_col", C.c_int32),
        ("fm_ld", C.c_int32), ("dx0_ld", C.c_int32), ("dx0_cat_col", C.c_int32), ("multi_width", C.c_int32),
        ("cont_rows_compact", C.c_int32), ("x0_bf16", C.c_int32),
    ]


class AdamLayer(C.Structure):
    """Mirror of ``dl_adam_layer`` (include/dlamd.h)."""
    _fields_ = [
        ("p", C.c_void_p), ("m", C.c_void_p), ("v", C.c_void_p), ("slab", C.c_void_p), ("slab_stride", C.c_int64),
        ("reg_count", C.c_int64), ("acc_out", C.c_void_p), ("wp", C.c_void_p), ("wtp", C.c_void_p),
        ("nslab", C.c_int32), ("rows", C.c_int32), ("cols", C.c_int32), ("reg_kind", C.c_int32), ("reg", C.c_float),
        ("pad_", C.c_int32)]


class PoolDesc(C.Structure):
    """Mirror of ``dl_pool_desc`` (include/dlamd.h)."""
    _fields_ = [
        ("slot_start", C.c_void_p), ("slot_end", C.c_void_p), ("n_slots", C.c_int32), ("fm_col", C.c_int32),
        ("dx0_pool_col", C.c_int32), ("g_pitch", C.c_int32), ("x0", C.c_void_p), ("cnt_emb", C.c_void_p),
        ("cnt_first", C.c_void_p), ("g_pool", C.c_void_p), ("g1_pool", C.c_void_p),
    ]


# include/dlamd.h constants
OPT_LEN, OPT_STATUS, OPT_SKIP, OPT_BAD_STEP, OPT_BAD_COUNT, OPT_SEQ, OPT_BAD_RANKS = 32, 16, 17, 18, 19, 20, 21
STATUS_BAD_ID, STATUS_LAG, STATUS_INDEX, STATUS_OVERFLOW, STATUS_DESYNC = 1, 2, 4, 8, 16
REC_FIRST, REC_SPARSE_ADAM, REC_PLANE_SLOTS = 1, 2, 4
ROWS_CLEAR_TOUCHED, ROWS_SPARSE_ADAM, ROWS_GRAD_FIXED = 1, 2, 4
WIDE_GRAD_SCALE = 2.0 ** 48
REG_SUM_SCALE = 2.0 ** 32   # int64 fixed-point regulariser sums (DL_REG_SUM_SCALE, opt[DL_OPT_REG])
OPT_REG = 8


def reg_sum(q):
    """A fixed-point regulariser sum (an int64 device or host tensor element, or the opt block:
    its opt[DL_OPT_REG..+1]) as a Python float."""
    import torch
    if q.dtype == torch.float32:
        q = q[OPT_REG: OPT_REG + 2].view(torch.int64)
    return int(q.reshape(-1)[0].item()) / REG_SUM_SCALE
LOSS_ACC_SLOTS = 65536

P = C.c_void_p
I32, I64, U64, F = C.c_int32, C.c_int64, C.c_uint64, C.c_float
LP = C.POINTER(EmbLayout)

# name -> (restype, argtypes); the authoritative list of exported entry points
SIGNATURES = {
    "dl_abi_version": (I32, []),
    "dl_last_error": (C.c_char_p, []),
    "dl_device_sync": (I32, []),
    "dl_embed_fwd": (I32, [LP, P, P, P, P, P, P, P, P, P, P]),
    "dl_embed_bwd": (I32, [LP, P, P, P, P, P, P, P, P, P, P, P, I32, P]),
    "dl_embed_bwd_grid": (I32, [LP]),
    "dl_embed_cont_reduce": (I32, [LP, P, I32, P, P, P, P]),
    "dl_embed_fwd_indexed": (I32, [LP, P, P, P, I32, P, P, P, P, P, P]),
    "dl_embed_fwd_slots": (I32, [LP, P, P, P, P, P, P, P, P, P]),
    "dl_embed_fwd_gtab": (I32, [LP, P, I32, P, P, P, P, P, P, P, P, P]),
    "dl_embed_fwd_gtab_ok": (I32, [LP]),
    "dl_embed_fwd_rec": (I32, [LP, P, I32, I32, P, P, P, P, P, P, I32, P, I32, P, P, P, P, P]),
    "dl_embed_fwd_rec_flat": (I32, [LP, P, I32, I32, P, P, P, P, P, P, P, P, P, P, P]),
    "dl_shard_gather": (I32, [P, P, P, I64, I32, P, P, P]),
    "dl_shard_scatter_add": (I32, [P, P, P, I64, I32, P, P, P, P]),
    "dl_shard_route": (I32, [P, P, P, I32, I32, I64, I32, P, P, P, P, P, P, I64, I64, P]),
    "dl_shard_stamp": (I32, [P, I32, I32, P, P]),
    "dl_shard_step_begin": (I32, [P, P, I32, I64, I64, P, F, F, P, I32, P]),
    "dl_slab_sum": (I32, [P, I32, I64, I64, P, P]),
    "dl_keys_to_local": (I32, [P, P, I64, P, P]),
    "dl_embed_cont_bwd": (I32, [LP, P, P, P, P, P, P, I32, P]),
    "dl_index_workspace_bytes": (I64, [I64]),
    "dl_index_build": (I32, [LP, P, I32, I32, P, I64, P, P, P, P, P, P, P, P, P]),
    "dl_index_build_pair": (I32, [LP, P, LP, P, P, I64, P, P, P, P, P, P, P, P, P, P, P, P, P]),
    "dl_embed_bwd_sorted": (I32, [LP, P, P, P, P, P, P, I32, I64, P, P, P, P, P, P, P, I32, P, P]),
    "dl_pool_fwd": (I32, [LP, P, P, P, I32, P, P, I32, I32, P, P, P, P, P, P]),
    "dl_pool_fwd_indexed": (I32, [LP, P, P, P, I32, P, P, I32, I32, P, P, P, P, P]),
    "dl_pool_bwd": (I32, [LP, P, I32, P, P, I32, I32, P, P, P, P, P, I32, P, P, P, P, P, P]),
    "dl_pool_fwd_weighted": (I32, [LP, P, P, I32, P, I32, P, P, I32, P, P, P, P]),
    "dl_pool_bwd_weighted": (I32, [LP, P, I32, P, I32, P, P, I32, P, I32, P, P, P, P]),
    "dl_gemm_f32": (I32, [I32, I32, I32, I32, I32, P, I32, P, I32, P, I32, I32, P, I32, I32, I64, P]),
    "dl_gemm_bf16": (I32, [I32, I32, I32, I32, I32, P, I32, P, I32, P, I32, I32, I32, P, I32, I32, I64, P]),
    "dl_split3": (I32, [P, I32, I32, I32, I32, P, I32, I64, P]),
    "dl_s3_kperm": (I32, []),
    "dl_gemm_s3_nt": (I32, [I32, I32, I32, P, I32, P, I32, I64, P, I32, I32, P, I32, P]),
    "dl_gemm_s3_nt_bits": (I32, [I32, I32, I32, P, I32, P, I32, I64, P, I32, I32, P, I32, P, I32, P]),
    "dl_gemm_s3_nt_gather": (I32, [I32, I32, I32, P, I32, P, I64, I32, P, I32, I64, I32, I32, I32, P, I32, I64, P,
                                   I32, I32, P, I32, P]),
    "dl_gemm_s3_nt_gather_rows": (I32, [I32, I32, I32, P, I32, P, I64, I32, P, I32, I32, I32, I32, P, I32, I64, P,
                                        I32, I32, P, I32, P]),
    "dl_gemm_s3_nt_gather_tab": (I32, [I32, I32, I32, P, I32, P, I64, I32, P, I32, I32, P, I32, I64, P, I32, I32,
                                       P, I32, P]),
    "dl_gemm_s3_tn": (I32, [I32, I32, I32, P, I32, P, I32, P, I32, I32, I64, P]),
    "dl_head_fwd_bwd": (I32, [I32, I32, I32, P, I32, P, I32, P, P, F, F, P, P, P, P, P, I32, P]),
    "dl_head_grid": (I32, [I32]),
    "dl_wdl_head_grid": (I32, [I32]),
    "dl_wdl_head_fwd_bwd": (I32, [I32, I32, I32, P, I32, P, I32, P, P, I64, P, F, F, P, P, P, P, P, P, P, I32, P, P]),
    "dl_wdl_head_fwd_bwd_bf16": (I32, [I32, I32, I32, P, I32, P, I32, P, P, I64, P, F, F, P, P, P, P, P, P, P, I32, P,
                                       P]),
    "dl_slab_fold_rows": (I32, [P, I32, I32, I32, I32, P, I64, P, P]),
    "dl_adam_begin_step": (I32, [P, F, F, P]),
    "dl_step_guard": (I32, [P, P, P]),
    "dl_step_begin": (I32, [P, P, F, F, P, I32, P]),
    "dl_loss_accumulate": (I32, [P, I32, I32, I32, C.c_double, P, F, P, P, P]),
    "dl_validate_batch": (I32, [LP, P, P, I32, I32, I64, I32, P, P]),
    "dl_adam_dense": (I32, [P, P, P, P, I32, I64, I64, F, I64, P, P, P, P]),
    "dl_adam_dense_split3": (I32, [P, P, P, P, I32, I64, I32, I32, F, I64, I32, P, P, P, P, P]),
    "dl_adam_dense_bf16": (I32, [P, P, P, P, I32, I64, I32, I32, F, I64, I32, P, P, P, P, P]),
    "dl_adam_dense_layers": (I32, [I32, P, I32, P, P]),
    "dl_adam_dense_reg": (I32, [P, P, P, P, I32, I64, I64, F, I64, I32, P, P, P, P]),
    "dl_adam_rows": (I32, [P, P, P, P, P, I64, I32, F, I32, P, P, P]),
    "dl_init_random": (I32, [P, I64, I32, F, F, U64, U64, P]),
    "dl_transpose_f32": (I32, [P, I32, I32, I32, P, I32, P]),
    "dl_cast_bf16": (I32, [P, I32, I32, I32, P, I32, P]),
    "dl_transpose_bf16": (I32, [P, I32, I32, I32, I32, P, I32, P]),
    "dl_adam_hist_record": (I32, [P, P, I32, P]),
    "dl_rec_stash_floats": (I32, [I32]),
    "dl_rec_gather": (I32, [LP, P, I32, I32, I32, P, P, I64, I32, P, I32, P, I32, P, P, P, P]),
    "dl_rec_gather_scatter": (I32, [LP, P, I32, I32, I32, P, P, I64, P, P, P, I32, P, I32, P, P, P, P, P, P, P, P, P]),
    "dl_pool_fwd_staged": (I32, [LP, P, P, P, P, P, I32, I32, P, P, P, P, P]),
    "dl_embed_fwd_staged": (I32, [LP, P, P, P, I32, P, P, P, P, P, P]),
    "dl_rec_bwd_adam": (I32, [LP, P, I32, I32, I32, P, P, P, P, P, P, P, I32, I64, P, P, P, P, P, P, P, I32, P,
                              P, P, I64, P]),
    "dl_rec_bwd_workspace_bytes": (I64, [I64, I32]),
    "dl_rec_apply_rows": (I32, [P, I32, I32, I32, I64, I64, P, P, P, I32, P, P]),
    "dl_sort_unique": (I32, [P, I64, I32, P, I64, P, P, P, P, P, P, P]),
    "dl_rec_apply_segments": (I32, [P, I32, I32, I32, P, P, P, I64, I64, P, P, P, P, P, P, P, I32, P, P]),
    "dl_rec_flush": (I32, [P, I32, I32, I32, I64, P, I32, P, P, P, P]),
    "dl_rec_chain_link": (I32, [P, I64, P, P, P]),
    "dl_rec_apply_chain": (I32, [P, I32, I32, I32, P, I64, P, P, P, P, P, I32, P, P]),
    "dl_auc_workspace_bytes": (I64, [I64]),
    "dl_auc": (I32, [P, I64, P, I64, I64, P, I64, P, P]),
    "dl_hbm_copy": (I32, [P, P, I64, P]),
    "dl_shard_gather_scalar": (I32, [P, P, I64, P, P]),
    "dl_shard_add_fixed": (I32, [P, P, I64, P, P, P]),
    "dl_wide_fold_owned": (I32, [P, I32, I64, I32, I32, P, P, P]),
    "dl_wide_owned_values": (I32, [P, I32, I64, I32, I32, P, P]),
    "dl_wide_local_ids": (I32, [P, I64, I64, P, P]),
    "dl_wide_rec_gather": (I32, [P, I64, P, P, I64, I32, I32, P, I32, P, F, I32, P, P, P, P]),
    "dl_wide_update_blocks": (I64, [I64, I32]),
    "dl_wide_seg_grad": (I32, [P, I32, P, P, P, I64, I64, P, P, P, P]),
    "dl_wide_rec_update": (I32, [P, P, I64, P, P, I32, I32, F, P, I32, P, P, P, P, P, P]),
    "dl_wide_rec_flush": (I32, [P, I64, F, P, I32, P, P, P, P]),
    "dl_comm_unique_id_bytes": (I32, []),
    "dl_comm_get_unique_id": (I32, [P]),
    "dl_comm_init": (I32, [P, I32, I32, P]),
    "dl_comm_destroy": (I32, [P]),
    "dl_all_to_allv": (I32, [P, P, P, P, P, I64, P]),
    "dl_all_reduce_f32": (I32, [P, P, P, I64, P]),
    "dl_all_gather": (I32, [P, P, P, I64, P]),
    "dl_shard_exchange": (I32, [P, I32, P, P, I32, P]),
}

_LIB = None


def lib():
    """Load (once) and return the ctypes library; raises if it is not built."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise DLError("libdlamd.so not found at %s — build it with `python -m deep_learning_amd.build`"
                          % LIB_PATH)
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _LIB = L
    return _LIB


def call(name, *args):
    rc = getattr(lib(), name)(*args)
    if rc != 0:
        raise DLError("%s failed (rc=%d): %s" % (name, rc, lib().dl_last_error().decode()))
    return rc


def ptr(t):
    """Device pointer of a torch tensor (None -> NULL)."""
    return None if t is None else C.c_void_p(t.data_ptr())


def stream_handle(stream=None):
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return C.c_void_p(s.cuda_stream)
