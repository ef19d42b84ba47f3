"""One-screen summary of a bench.py JSON line: headline, roofline, CPU baseline, the extra
workloads and the slowest kernels of each.  usage: python scripts/bench_brief.py bench.json"""
import json
import sys


def kernels(k, n=8):
    top = sorted(k.items(), key=lambda kv: -kv[1].get("us", 0))[:n]
    return "  ".join("%s %.0f" % (name, v.get("us", 0)) for name, v in top)


def main(path):
    d = json.loads(open(path).read().strip().splitlines()[-1])
    print("%s: %.4f ms/step, %.3g samples/s, n_gpus %s, %s, world %s" % (
        d["config"]["workload"], d["ms_per_step"], d["value"], d["n_gpus"], d["config"]["parallelism"], d.get("world")))
    r = d["roofline"]
    print("  roofline %s %s: %.4g %s = %.3f of peak, traffic %s" % (
        r.get("kernel"), r["bound"], r["achieved"], r["unit"], r["frac"], r.get("traffic")))
    print("  kernels(us): " + kernels(d["kernels"]))
    if d.get("cpu_baseline"):
        c = d["cpu_baseline"]
        print("  cpu baseline: %s %s (%s cores, %s)" % (c.get("value"), c.get("unit"), c.get("cores"), c.get("sample")))
    for w, e in (d.get("extra_workloads") or {}).items():
        if "error" in e:
            print("  %s: ERROR %s" % (w, e["error"]))
            continue
        print("  %s: %.4f ms/step, %.3g samples/s; %s" % (w, e["ms_per_step"], e["samples_per_s"], kernels(e["kernels"])))


if __name__ == "__main__":
    main(sys.argv[1])
