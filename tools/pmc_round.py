"""Reduces tools/pmc_round.sh's passes into profiles/<tag>_pmc_<kernel>.json: per-call counter values
per page for the C2 LZ4 kernels (encode: 2 dispatches per run, decode: 1), the derived ratios, and the
kernel-source digest and commit they were taken on.

    python tools/pmc_round.py gpurun_out/pmc_r04 r04 [pages]
"""
import csv
import glob
import json
import os
import subprocess
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tyche_amd._build import kernel_sources_digest  # noqa: E402

KERNELS = {"lz4_decode": "lz4_decode_lc_kernel", "lz4_encode": "lz4_encode_splitn_kernel"}


def main():
    d, tag = sys.argv[1], sys.argv[2]
    pages = int(sys.argv[3]) if len(sys.argv) > 3 else 262144
    acc = {k: defaultdict(float) for k in KERNELS}
    disp = {k: defaultdict(set) for k in KERNELS}
    for f in glob.glob(os.path.join(d, "*", "run_counter_collection.csv")):
        pas = os.path.basename(os.path.dirname(f))
        for r in csv.DictReader(open(f)):
            for k, sym in KERNELS.items():
                if sym in r["Kernel_Name"]:
                    acc[k][r["Counter_Name"] + "@" + pas] += float(r["Counter_Value"])
                    disp[k][pas].add(r["Dispatch_Id"])
    head = subprocess.run(["git", "-C", ROOT, "rev-parse", "--short=12", "HEAD"], capture_output=True,
                          text=True).stdout.strip()
    for k in KERNELS:
        if not acc[k]:
            continue
        per = {}
        for key, v in acc[k].items():
            name, pas = key.split("@")
            n = len(disp[k][pas])
            per.setdefault(name, {})[pas] = v / n / pages     # per call, per page
        vals = {name: round(sum(x.values()) / len(x), 2) for name, x in per.items()}
        wc = vals.get("SQ_WAVE_CYCLES")
        gui = vals.get("GRBM_GUI_ACTIVE")
        derived = {}
        if wc:
            for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY"):
                if c in vals:
                    derived[c + "_per_wave_quad_cycle"] = round(vals[c] / wc, 4)
        if gui:   # per-CU units summed over 256 CUs, GRBM over 8 XCDs: fraction of the kernel's cycles
            for c in ("TA_TA_BUSY", "TD_TD_BUSY", "TD_TC_STALL", "TCP_PENDING_STALL_CYCLES", "SQ_LDS_IDX_ACTIVE",
                      "SQ_LDS_BANK_CONFLICT"):
                if c in vals:
                    derived[c + "_frac_of_cu_cycles"] = round(vals[c] / 256.0 / (gui / 8.0), 3)
        if "TCC_EA0_RDREQ_sum" in vals and "TCP_TCC_READ_REQ" in vals:
            derived["l2_read_miss_frac"] = round(vals["TCC_EA0_RDREQ_sum"] / vals["TCP_TCC_READ_REQ"], 3)
        out = {"kernel": KERNELS[k], "pages_per_call": pages, "page_len": 16384, "per_page_per_call": vals,
               "derived": derived, "kernel_sources_sha16": kernel_sources_digest(), "commit": head,
               "source": "tools/pmc_round.sh over tools/run_codec.py (REPS=1), rocprofv3 --pmc, one pass per set"}
        p = os.path.join(ROOT, "profiles", f"{tag}_pmc_{k}.json")
        json.dump(out, open(p, "w"), indent=1)
        print(p, json.dumps(derived))


if __name__ == "__main__":
    main()
