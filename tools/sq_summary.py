#!/usr/bin/env python3
"""Summarise the SQ/LDS/VALU counter passes of scripts/gpu_sq.sh
(gpurun_out/sq_<w>_<pass>/) for each workload's kernels: per-launch medians
and the derived shares that say what binds a kernel (VALU-active vs
LDS-active vs waiting). SQ cycle counters are quad-cycles summed over SEs
(MI355X_MICROARCH.md, s_memtime row); the ratios below are unit-free."""
import csv
import glob
import json
import os
import statistics
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def collect(w):
    vals = defaultdict(lambda: defaultdict(list))
    for path in sorted(glob.glob(os.path.join(REPO, "gpurun_out", f"sq_{w}_*", "run_counter_collection.csv"))):
        for r in csv.DictReader(open(path)):
            k = r["Kernel_Name"].split("(")[0]
            if "fill_uniform" in k:
                continue
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            vals[k]["_vgpr"] = [float(r["VGPR_Count"])]
            vals[k]["_lds"] = [float(r["LDS_Block_Size"])]
    out = {}
    for k, d in vals.items():
        m = {c: statistics.median(v) for c, v in d.items()}
        wc = m.get("SQ_WAVE_CYCLES") or 1
        busy = m.get("SQ_BUSY_CYCLES") or 1
        m["share_active_valu"] = m.get("SQ_ACTIVE_INST_VALU", 0) / wc
        m["share_active_lds"] = m.get("SQ_ACTIVE_INST_LDS", 0) / wc
        m["share_wait_any"] = m.get("SQ_WAIT_ANY", 0) / wc
        m["share_wait_inst_any"] = m.get("SQ_WAIT_INST_ANY", 0) / wc
        m["share_wait_inst_lds"] = m.get("SQ_WAIT_INST_LDS", 0) / wc
        m["lds_bank_conflict_per_active"] = m.get("SQ_LDS_BANK_CONFLICT", 0) / max(1, m.get("SQ_LDS_IDX_ACTIVE", 1))
        f64 = 2 * m.get("SQ_INSTS_VALU_FMA_F64", 0) + m.get("SQ_INSTS_VALU_ADD_F64", 0) + m.get("SQ_INSTS_VALU_MUL_F64", 0)
        m["f64_flop"] = 64 * f64
        m["f64_inst_share_of_valu"] = (m.get("SQ_INSTS_VALU_FMA_F64", 0) + m.get("SQ_INSTS_VALU_ADD_F64", 0)
                                       + m.get("SQ_INSTS_VALU_MUL_F64", 0)) / max(1, m.get("SQ_INSTS_VALU", 1))
        # the VALU pipe's busy share: every wave64 VALU instruction holds a
        # 16-lane SIMD for 4 cycles; GRBM_GUI_ACTIVE is summed over the 8 XCDs
        # (MI355X_MICROARCH.md), each XCD 32 CUs x 4 SIMDs
        if m.get("GRBM_GUI_ACTIVE"):
            m["valu_pipe"] = 4 * m.get("SQ_INSTS_VALU", 0) / (m["GRBM_GUI_ACTIVE"] / 8 * 1024)
        out[k] = m
    return out


def main(tag, workloads):
    res = {w: collect(w) for w in workloads}
    if tag == "-":  # print only (experiments)
        merged = None
    dst = os.path.join(REPO, "profiles", tag)
    if tag != "-":
        os.makedirs(dst, exist_ok=True)
        path = os.path.join(dst, "sq_counters.json")
        merged = json.load(open(path)) if os.path.exists(path) else {}
        merged.update(res)  # the workloads re-measured replace their entries
        with open(path, "w") as f:
            json.dump(merged, f, indent=1, sort_keys=True)
    for w, ks in res.items():
        print("==", w)
        for k, m in ks.items():
            print(f"  {k[:60]:60s} vgpr={m['_vgpr']:.0f} lds={m['_lds']:.0f} valu={m['share_active_valu']:.2f} "
                  f"lds={m['share_active_lds']:.2f} wait={m['share_wait_any']:.2f} "
                  f"waitinst={m['share_wait_inst_any']:.2f} waitlds={m['share_wait_inst_lds']:.2f} "
                  f"bankconf={m['lds_bank_conflict_per_active']:.3f} f64flop={m['f64_flop']:.3e} "
                  f"insts valu={m.get('SQ_INSTS_VALU',0):.3e} lds={m.get('SQ_INSTS_LDS',0):.3e} "
                  f"salu={m.get('SQ_INSTS_SALU',0):.3e} vmem={m.get('SQ_INSTS_VMEM',0):.3e} "
                  f"grbm={m.get('GRBM_GUI_ACTIVE',0):.3e} waves={m.get('SQ_WAVES',0):.3e} "
                  f"wavecyc={m.get('SQ_WAVE_CYCLES',0):.3e} busy={m.get('SQ_BUSY_CYCLES',0):.3e}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r01",
         sys.argv[2:] or ["radix4096", "bluestein3000", "chirpz3000", "pwelch", "fft2_8192"])
