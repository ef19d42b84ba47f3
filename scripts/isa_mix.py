"""Static instruction mix of a kernel in a HIP source's gfx950 assembly, split into the main
loop (the blocks between the loop header and its back edge) and the rest (prologue +
epilogue): how many non-MFMA VALU instructions a chunk of MFMAs carries, by opcode.
    python scripts/isa_mix.py deep_learning_amd/csrc/gemm.hip <kernel-symbol-substring>"""
import collections
import os
import re
import subprocess
import sys
import tempfile

src, pat = sys.argv[1], sys.argv[2]
here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
out = os.path.join(tempfile.mkdtemp(), "k.s")
subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-S", "--cuda-device-only",
                "-I" + os.path.join(here, "include"), "-I" + os.path.join(here, "deep_learning_amd", "csrc"),
                src, "-o", out], check=True, stderr=subprocess.DEVNULL)
s = open(out).read()
names = [n for n in re.findall(r"^(\S+):\s*;\s*@", s, re.M) if pat in n]
for name in names:
    i = s.index(name + ":")
    j = s.index(".Lfunc_end", i)
    body = s[i:j].splitlines()
    # the loop: from the first "Loop Header" label to the last branch back to it
    hdr = next((n for n, l in enumerate(body) if "Loop Header" in l), None)
    lab = body[hdr].split(":")[0].strip() if hdr is not None else None
    back = max((n for n, l in enumerate(body) if lab and re.search(r"s_c?branch\w*\s+" + re.escape(lab) + r"\b", l)),
               default=None)
    def mix(lines):
        c = collections.Counter()
        for l in lines:
            t = l.strip()
            if not t or t.startswith((".", ";")) or t.endswith(":"):
                continue
            c[t.split()[0]] += 1
        return c
    loop = mix(body[hdr:back + 1]) if back else collections.Counter()
    rest = mix(body[:hdr] + body[back + 1:]) if back else mix(body)
    def summ(c, tag):
        mfma = sum(v for k, v in c.items() if "mfma" in k)
        valu = {k: v for k, v in c.items() if k.startswith("v_") and "mfma" not in k}
        print("  %s: %d MFMA, %d non-MFMA VALU (%.2f a MFMA), %d s_waitcnt, %d VMEM, %d LDS" % (
            tag, mfma, sum(valu.values()), sum(valu.values()) / max(mfma, 1), c["s_waitcnt"],
            sum(v for k, v in c.items() if k.startswith(("buffer_", "global_"))),
            sum(v for k, v in c.items() if k.startswith("ds_"))))
        print("    " + ", ".join("%s %d" % kv for kv in sorted(valu.items(), key=lambda kv: -kv[1])[:14]))
    print(name)
    summ(loop, "main loop (static)")
    summ(rest, "prologue + epilogue (static)")
