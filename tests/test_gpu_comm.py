"""The C ABI's RCCL entry points (comm.cpp) on one GPU: a one-rank
communicator, so every collective's result is known exactly (all-to-allv to self is a copy,
the sum over one rank is the input, the all-gather of one rank is the input)."""
import ctypes

import pytest
import torch

from deep_learning_amd import _lib


@pytest.mark.gpu
def test_rccl_entry_points_single_rank(hip_lib):
    L = _lib.lib()
    uid = ctypes.create_string_buffer(L.dl_comm_unique_id_bytes())
    assert L.dl_comm_get_unique_id(uid) == 0, L.dl_last_error()
    comm = ctypes.c_void_p()
    assert L.dl_comm_init(uid, 1, 0, ctypes.byref(comm)) == 0, L.dl_last_error()
    s = _lib.stream_handle()
    try:
        # rows of 17 floats (68 B: the row exchange of an E=16 row + first-order weight)
        x = torch.randn(1000, 17, device="cuda")
        y = torch.full_like(x, float("nan"))
        cnt = (ctypes.c_int64 * 1)(1000)
        assert L.dl_all_to_allv(comm, _lib.ptr(x), cnt, _lib.ptr(y), cnt, 17 * 4, s) == 0, L.dl_last_error()
        r = torch.randn(5001, device="cuda")
        r0 = r.clone()
        assert L.dl_all_reduce_f32(comm, _lib.ptr(r), _lib.ptr(r), r.numel(), s) == 0, L.dl_last_error()
        g = torch.arange(9, dtype=torch.int64, device="cuda")
        go = torch.empty_like(g)
        assert L.dl_all_gather(comm, _lib.ptr(g), _lib.ptr(go), g.numel() * 8, s) == 0, L.dl_last_error()
        torch.cuda.synchronize()
        assert torch.equal(x, y)
        assert torch.equal(r, r0)
        assert torch.equal(g, go)
        # argument errors come back as codes with a message, nothing launched
        bad = (ctypes.c_int64 * 1)(-1)
        assert L.dl_all_to_allv(comm, _lib.ptr(x), bad, _lib.ptr(y), bad, 4, s) == 22
        assert b"negative" in L.dl_last_error()
    finally:
        assert L.dl_comm_destroy(comm) == 0
