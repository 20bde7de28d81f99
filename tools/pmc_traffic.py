"""Per-launch HBM traffic of the coverage kernels from two rocprofv3 --pmc passes.

    python tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write --config 4 \
        --out profiles/pmc_traffic_config4.json

FETCH_SIZE and WRITE_SIZE are collected in separate passes (gfx950 cannot fit both in one
pass) with --kernel-trace-free counter collection only. Corrections, per
/opt/skills/guides/MI355X_MICROARCH.md "HBM [CDNA4]":
  * the counters are in KiB (rocprofv3 derived metrics: TCC_EA0_*REQ x 64 B / 1024);
  * on gfx950 FETCH_SIZE reports 1/2 of the bytes of wide coalesced reads, so it is doubled;
  * Infinity-Cache hits are counted by the memory-side counters, not excluded.
Per kernel: 2 * FETCH + WRITE averaged over its launches (and, uncorrected, FETCH + WRITE: the
doubling is calibrated for 16-B-per-lane streaming reads only, so for gather- and hash-heavy
kernels the corrected figure is an upper bound and the raw one a lower bound; both are kept,
per kernel and per poll). "hbm_bytes_per_poll" sums the kernels
of one poll chain (--chain; the default launch chain by default), which bench.py reports as
roofline.traffic — only while the library sources hash to "src_sha" (bench.src_hash), i.e. the
build that was profiled. Run the passes with `bench.py --no-extras` so that only the poll chain
launches after set-up.
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import json
import os


def load(d: str, counter: str):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    per = collections.defaultdict(list)
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row["Counter_Name"] != counter:
                    continue
                name = row["Kernel_Name"].split("(")[0].replace("void ", "")
                per[name].append(float(row["Counter_Value"]))
    return per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--config", type=int, default=4)
    ap.add_argument("--chain", default="mac::prep_x_kernel<false>;mac::fiw_kernel<true>;mac::fin2_kernel<true>",
                    help="semicolon-separated kernels of one poll (default: the fused chain "
                         "config 4 takes; the five-launch chain: mac::prep_kernel;"
                         "mac::disk_index_kernel<true, 3>;mac::walk_setup_kernel;"
                         "mac::coverage_poll_kernel;mac::finalize_kernel)")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    fetch = load(a.fetch_dir, "FETCH_SIZE")
    write = load(a.write_dir, "WRITE_SIZE")
    kernels = {}
    for name in sorted(set(fetch) | set(write)):
        f = fetch.get(name, [])
        w = write.get(name, [])
        if not f or not w:
            continue
        fk = sum(f) / len(f)
        wk = sum(w) / len(w)
        kernels[name] = {
            "launches": len(f),
            "fetch_kib_raw": fk,
            "write_kib_raw": wk,
            "hbm_bytes_per_launch": 2.0 * fk * 1024.0 + wk * 1024.0,
            "hbm_bytes_per_launch_raw": fk * 1024.0 + wk * 1024.0,
        }
    chain = a.chain.split(";")
    missing = [k for k in chain if k not in kernels]
    if missing:
        raise SystemExit(f"{missing} not found; have {list(kernels)}")
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    out = {
        "config": a.config,
        "workload": "bench.py default (uniform disks, cons3, algo auto)",
        "src_sha": bench.src_hash(),
        "chain": chain,
        "hbm_bytes_per_poll": sum(kernels[k]["hbm_bytes_per_launch"] for k in chain),
        "hbm_bytes_per_poll_raw": sum(kernels[k]["hbm_bytes_per_launch_raw"] for k in chain),
        "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over "
                  "`python3 bench.py --steps 5 --warmup 1 --no-cpu --no-extras`; bytes = "
                  "2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 FETCH correction, "
                  "MI355X_MICROARCH.md: calibrated for wide streaming reads, so an upper bound "
                  "for gathers); *_raw = FETCH_SIZE*1024 + WRITE_SIZE*1024 (a lower bound)",
        "kernels": kernels,
    }
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps({k: round(v["hbm_bytes_per_launch"] / 1e6, 3) for k, v in kernels.items()},
                     indent=1))


if __name__ == "__main__":
    main()
