"""The north-star lookup alone (C2 shape, B = 65,536, 26 M rows): dl_embed_fwd over the dense
p / first-order planes of a flushed table, the kernel CTREngine.predict runs — nothing else
launches embed_fwd_kernel here (no training step), so rocprofv3 PMC passes over this script
count the lookup alone.  python scripts/lookup_bench.py [uniform|zipf] [reps] [full|fm|fused|pair|fmtab|tab]
(fm: the FM-only lookup of the fused predict, x0_cat_col = -1 — the deep rows are then read by
dl_gemm_s3_nt_gather, not here; fused: that lookup + the gathering first tower layer, predict's
id form; pair: the full lookup + the plain first layer, the unfused front; fmtab: the lookup of
the table form, dl_embed_fwd_gtab — FM outputs, x0's cont columns and the deep rows' plane
offsets; tab: that + dl_gemm_s3_nt_gather_tab, predict's front with DLAMD_GATHER_TAB=1)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deep_learning_amd import _lib  # noqa: E402
from deep_learning_amd._lib import call, ptr  # noqa: E402
from deep_learning_amd.engine import C_ref, CTREngine, ModelSpec  # noqa: E402
from deep_learning_amd.synthetic import make_batch  # noqa: E402

dist = sys.argv[1] if len(sys.argv) > 1 else "uniform"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
mode = sys.argv[3] if len(sys.argv) > 3 else "full"
B, N = 65536, 26_000_000
spec = sp = ModelSpec("deepfm_pipeline", C=13, V=0, S=26, E=16, cate_index_size=N, hidden=[400, 400, 400])
eng = CTREngine(spec, max_batch=B, seed=2019, adam="lazy")
eng.flush(planes=True)
b = {k: torch.from_numpy(v).cuda() for k, v in make_batch(B, cate_index_size=N, seed=4242, dist=dist).items()}
eng.stage(b)
FL = eng._flat_layout(B)
FN = eng._flat_layout(B)
FN.x0_cat_col = -1
if mode in ("fm", "fused"):
    FL = FN
tab = mode in ("fmtab", "tab")
if tab:
    assert eng.fused_gather_tab(B, force=True)
hd, ld0, ol0 = sp.hidden[0], eng.in_ld[0], eng.out_ld[0]
bits = (ptr(eng.hbits[0]), eng.hbits_ld[0]) if eng.hbits else (None, 0)


def layer0():
    if mode == "fused":
        call("dl_gemm_s3_nt_gather", B, hd, ld0, ptr(x0), ld0, ptr(eng.p_plane), FN.n_rows, eng.p_plane.shape[1],
             ptr(eng.in_cate), FN.cate_ld, FN.deep_cate_offset, FN.zero_row0, sp.S, sp.E, ptr(eng.WTp[0]), ld0,
             ld0 * ol0, ptr(eng.h[0]), eng.h_ld[0], 1, *bits, s)
    elif mode == "tab":
        call("dl_gemm_s3_nt_gather_tab", B, hd, ld0, ptr(x0), ld0, ptr(eng.p_plane), FN.n_rows, eng.p_plane.shape[1],
             ptr(eng.gtab), sp.S, sp.E, ptr(eng.WTp[0]), ld0, ld0 * ol0, ptr(eng.h[0]), eng.h_ld[0], 1, *bits, s)
    elif mode == "pair":
        call("dl_gemm_s3_nt_bits", B, hd, ld0, ptr(x0), ld0, ptr(eng.WTp[0]), ld0, ld0 * ol0, ptr(eng.h[0]),
             eng.h_ld[0], 1, None, 0, *bits, s)
s = _lib.stream_handle()
x0 = eng.x0b if eng.x0_direct else eng.x0


def run():
    if tab:
        call("dl_embed_fwd_gtab", C_ref(FN), ptr(eng.p_plane), 1, ptr(eng.in_cate), ptr(eng.in_cont), ptr(eng.in_vec),
             ptr(x0), ptr(eng.fm_out), None, ptr(eng.gtab), ptr(eng.err), s)
    elif sp.fm:   # the slot plane: an FM reference's row and first-order weight in one 128-B slot
        call("dl_embed_fwd_slots", C_ref(FL), ptr(eng.p_plane), ptr(eng.in_cate), ptr(eng.in_cont), ptr(eng.in_vec),
             ptr(x0), ptr(eng.fm_out), ptr(eng.fm_sum), ptr(eng.err), s)
    else:
        call("dl_embed_fwd", C_ref(FL), ptr(eng.p_plane), None, ptr(eng.in_cate), ptr(eng.in_cont),
             ptr(eng.in_vec), ptr(x0), ptr(eng.fm_out), ptr(eng.fm_sum), ptr(eng.err), s)
    layer0()


run()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(reps):
    run()
e1.record()
torch.cuda.synchronize()
eng.check_error()
us = e0.elapsed_time(e1) * 1e3 / reps
print("lookup %s %s %.1f us  %.3f of 8 TB/s by the 3,640-B rule" % (mode, dist, us, B * 3640 / us / 1e3 / 8000), flush=True)
