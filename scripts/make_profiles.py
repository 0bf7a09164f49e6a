"""Copy a scripts/gpu_prof.sh run into the tracked profiles/ directory.

usage: python scripts/make_profiles.py gpurun_out/prof_<tag> <round_tag>

Writes profiles/<round_tag>_kernel_stats.csv (rocprofv3 --kernel-trace --stats summary),
profiles/<round_tag>_summary.txt (per-kernel avg duration + PMC bytes per launch) and
profiles/pmc_traffic.json (HBM bytes per launch = 2*FETCH_SIZE + WRITE_SIZE, KiB->B, the gfx950
FETCH_SIZE correction of MI355X_MICROARCH.md §HBM), which bench.py reads for roofline.traffic.
"""
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    src, tag = sys.argv[1], sys.argv[2]
    out = os.path.join(ROOT, "profiles")
    os.makedirs(out, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"),
                os.path.join(out, tag + "_kernel_stats.csv"))
    txt = subprocess.check_output([sys.executable, os.path.join(ROOT, "scripts", "summarize_prof.py"),
                                   src]).decode()
    bench = os.path.join(os.path.dirname(src), os.path.basename(src) + ".bench.json")
    hdr = ("# rocprofv3 --kernel-trace --stats + separate --pmc passes (FETCH_SIZE | WRITE_SIZE |\n"
           "# TCC_HIT_sum TCC_MISS_sum | GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES) of\n"
           "#   python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-wavenet\n"
           "# (scripts/gpu_prof.sh).  FETCH_KB/WRITE_KB are raw counter values per launch (KiB);\n"
           "# HBM bytes = 2*FETCH + WRITE on gfx950.  clk_GHz column is not meaningful.\n")
    with open(os.path.join(out, tag + "_summary.txt"), "w") as f:
        f.write(hdr + txt)
        if os.path.exists(bench):
            f.write("\n# bench line of the traced run:\n" + open(bench).read())
    summ = json.load(open(os.path.join(src, "summary.json")))
    kernels = {}
    groups = {}
    for k, v in summ.items():
        base = k.split("<")[0]
        if v.get("hbm_bytes_per_launch") is None:
            continue
        kernels[k] = dict(avg_us=v["avg_us"], calls=v["calls"],
                          hbm_bytes_per_launch=v["hbm_bytes_per_launch"])
        groups.setdefault(base, []).append(v)
    for base, vs in groups.items():
        if base in kernels:
            continue
        n = sum(v["calls"] for v in vs)
        kernels[base] = dict(
            avg_us=sum(v["avg_us"] * v["calls"] for v in vs) / n, calls=n,
            hbm_bytes_per_launch=sum(v["hbm_bytes_per_launch"] * v["calls"] for v in vs) / n,
            note="call-weighted mean over template instances " + ", ".join(
                k for k in summ if k.split("<")[0] == base))
    json.dump(dict(source=tag, method="2*FETCH_SIZE+WRITE_SIZE per launch (KiB->bytes), separate "
                   "--pmc passes", kernels=kernels),
              open(os.path.join(out, "pmc_traffic.json"), "w"), indent=1)
    print(open(os.path.join(out, tag + "_summary.txt")).read())


if __name__ == "__main__":
    main()
