#!/usr/bin/env python3
"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (gpurun_out/pmc_<w>_<C>/)
into profiles/pmc_<w>.json: HBM bytes per launch of the workload's dominant
kernel. Units and gfx950 correction per MI355X_MICROARCH.md §HBM: counters are
in KiB; FETCH_SIZE reports half the bytes of a 16-B/lane streaming read, so it
is doubled; WRITE_SIZE is exact for 16-B/lane stores."""
import csv
import json
import os
import shutil
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = {"radix4096": "fft_lds_kernel<12", "bluestein3000": "fft_mixed_fixed_kernel",
           "chirpz3000": "chirpz6k_kernel",
           "pwelch": "pwelch_row_kernel<12",
           "pwelch_default": "pwelch_wave_kernel<8",
           "prime3001": "rader_fixed_kernel",
           "pfa3027": "rader_pfa_kernel",
           # one FFT2 step = row pass + the two column-tile launches: summed
           "fft2_8192": ["fft_lds_kernel<13", "colfft_tile_kernel<7", "colfft_tile_kernel<6"],
           # one FFTN step = the row pass + two column-tile axes
           "fftn_512": ["fft_lds_kernel<9", ("colfft_tile_kernel<9", 2)],
           "wav_decode": "wav_decode_vec_kernel",
           # one 2^20 four-step at batch 1: column tiles (256), rows of 4096, transpose
           "fft_2p20": ["colfft_tile_kernel<8", "fft_lds_kernel<12", "transpose_kernel"]}


def session_stamp():
    """The sources the PMC session ran on (gpurun_out/source_stamp.json,
    written on the GPU box by the session script: tools/source_stamp.py)."""
    p = os.path.join(REPO, "gpurun_out", "source_stamp.json")
    if not os.path.exists(p):
        return None
    with open(p) as f:
        return json.load(f)


def values(w, counter, kernel):
    path = os.path.join(REPO, "gpurun_out", f"pmc_{w}_{counter}", "run_counter_collection.csv")
    rows = [r for r in csv.DictReader(open(path)) if kernel in r["Kernel_Name"]]
    return [float(r["Counter_Value"]) for r in rows], path


def main(w, tag):
    ks = KERNELS[w] if isinstance(KERNELS[w], list) else [KERNELS[w]]
    f_kib = w_kib = 0.0
    fetch = write = []
    for k in ks:
        k, mult = k if isinstance(k, tuple) else (k, 1)  # launches of k per step
        fetch, pf = values(w, "FETCH_SIZE", k)
        write, pw = values(w, "WRITE_SIZE", k)
        f_kib += mult * statistics.median(fetch)
        w_kib += mult * statistics.median(write)
    out = {
        "workload": w, "kernel": KERNELS[w], "launches": [len(fetch), len(write)],
        "fetch_size_kib": f_kib, "write_size_kib": w_kib,
        "hbm_read_bytes_per_launch": int(2 * f_kib * 1024),
        "hbm_write_bytes_per_launch": int(w_kib * 1024),
        "hbm_bytes_per_launch": int((2 * f_kib + w_kib) * 1024),
        "correction": "FETCH_SIZE x2 (gfx950 16-B/lane streaming reads), KiB -> bytes",
        "source": f"profiles/{tag}/pmc_{w}_FETCH_SIZE.csv, profiles/{tag}/pmc_{w}_WRITE_SIZE.csv",
        "stamp": session_stamp(),
    }
    dst = os.path.join(REPO, "profiles", tag)
    os.makedirs(dst, exist_ok=True)
    shutil.copy(pf, os.path.join(dst, f"pmc_{w}_FETCH_SIZE.csv"))
    shutil.copy(pw, os.path.join(dst, f"pmc_{w}_WRITE_SIZE.csv"))
    with open(os.path.join(REPO, "profiles", f"pmc_{w}.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    for w in sys.argv[2:]:
        main(w, sys.argv[1])
