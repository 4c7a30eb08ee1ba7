"""Reduces a rocprofv3 --pmc counter_collection.csv (tools/pmc_sq.sh) to per-kernel sums and per-page
figures, plus the derived issue fractions (VALU / SALU / LDS instructions per wave-cycle).

    python tools/pmc_sq_reduce.py gpurun_out/pmc_sq/.../run_counter_collection.csv --pages 65536 [-k lz4_decode]
"""
import argparse
import csv
import json
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--pages", type=int, required=True)
    ap.add_argument("-k", "--kernel", default="", help="substring of the kernel names to keep")
    a = ap.parse_args()
    acc = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for r in csv.DictReader(open(a.csv)):
        name = r["Kernel_Name"].replace("(anonymous namespace)", "anon").split("(")[0]
        if a.kernel not in name:
            continue
        acc[name][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[name].add(r["Dispatch_Id"])
    for name, c in acc.items():
        out = {"kernel": name, "dispatches": len(disp[name]), "pages": a.pages,
               "per_page": {k: round(v / a.pages, 1) for k, v in sorted(c.items())}}
        wc = c.get("SQ_WAVE_CYCLES")
        if wc:
            for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY",
                      "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
                if k in c:
                    out.setdefault("per_wave_cycle", {})[k] = round(c[k] / wc, 4)
        print(json.dumps(out))


if __name__ == "__main__":
    main()
