#!/usr/bin/env python3
"""Turns two rocprofv3 --pmc passes (FETCH_SIZE and WRITE_SIZE, each its own
run, --kernel-trace only) into profiles/pmc_latest.json: HBM bytes per launch
and per record for each kernel of interest.

Units and gfx950 corrections follow MI355X_MICROARCH.md (HBM / rocprofv3):
FETCH_SIZE and WRITE_SIZE are in KiB; FETCH_SIZE reports half the bytes of a
16-byte-per-lane streaming read, WRITE_SIZE is exact for 16-byte stores, and
other widths are uncalibrated. We therefore calibrate every access width we
use on the copy kernels of tools/copy_ceiling.hip (1 GiB read + 1 GiB written,
launched by tools/pmc_calib.py in the same passes) and scale each kernel's
counters by the factor of the access width it issues:

  plan_binary_decode_kernel : reads 16 B/lane (LDS-DMA), writes 8 B/lane
  plan_binary_encode_kernel : reads 8 B/lane, writes 16 B/lane

usage: pmc_summary.py PMC_ROOT RECORDS_PER_LAUNCH [OUT.json]   (config 2's plan kernels)
       pmc_summary.py PMC_ROOT --config C [--nested] [--out OUT.json]
                     (tools/profile_round.sh: every kernel of config C, or of its nested leg,
                      -> OUT.json, default profiles/pmc_cC.json)
  PMC_ROOT holds fetch_calib/, write_calib/ (pmc_calib.py) and fetch_bench/,
  write_bench/ (bench.py) rocprofv3 output directories.
"""
import csv
import glob
import json
import os
import sys

CALIB_BYTES = 1 << 30
WIDTHS = {"plan_binary_decode_kernel": (16, 8), "plan_binary_encode_kernel": (8, 16)}
ALGO = {"plan_binary_decode_kernel": 89 + 72, "plan_binary_encode_kernel": 64 + 89}


def load(d, counter):
    """kernel short name -> list of per-dispatch counter values (KiB)."""
    out = {}
    files = glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True)
    if not files:
        raise SystemExit("no counter_collection csv under %s" % d)
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                name = row["Kernel_Name"].replace("(anonymous namespace)::", "")
                name = name.replace("void ", "").split("(")[0].split("<")[0].split("::")[-1]
                out.setdefault(name, []).append(float(row["Counter_Value"]))
    return out


def main_config(root, config, out_path=None, nested=False):
    """Every kernel of one bench config (tools/profile_round.sh): all of them
    read their input with 16-byte LDS-DMA / vector loads and store 16-byte
    vectors (offsets: 8-byte stores, same calibration factors), so the 16-byte
    factors apply. Records per launch and the decode / encode kernels'
    algorithmic bytes come from the bench line of the FETCH pass; with
    `nested` from its nested leg (bench.py --nested: the nested programs'
    records and algorithmic bytes per call). The summary is stamped with the
    kernel-source hash (tools/srchash.py) and GIT_COMMIT, so bench.py can refuse
    it once the kernels change."""
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    from srchash import source_hash

    if out_path is None:
        out_path = os.path.join(os.path.dirname(here), "profiles", "pmc_c%d.json" % config)
    line = None
    with open(os.path.join(root, "fetch_bench.log")) as fh:
        for ln in fh:
            if ln.startswith("{") and '"metric"' in ln:
                line = json.loads(ln)
    if line is None:
        raise SystemExit("no bench line in fetch_bench.log")
    if nested:
        nl = line["nested"]
        n = nl["records"]
        wire, rec = nl["wire_bytes"] / n, nl["record_bytes"]
        a = nl["roofline"]["algorithmic_bytes_per_call"] / n
        algo = {"tgpu_jit_ndecode": a, "tgpu_jit_nwrite": a}
        calls = {"decode_call": ("tgpu_jit_ndecode", a),
                 "encode_call": ("tgpu_jit_nsize+tgpu_jit_nwrite", a)}
    else:
        n = line["config"]["records_per_gpu"]
        wire = line["config"]["wire_bytes_per_record"]
        rec = line["config"]["record_bytes"]
        roof = line["roofline"]
        algo = {}
        # a call's kernels joined by '+': the call's bytes go to its main kernel
        algo[roof["kernel"].split("+")[-1]] = roof["algorithmic_bytes_per_launch"] / n
        if "encode" in roof:
            algo[roof["encode"]["kernel"].split("+")[-1]] = \
                roof["encode"]["algorithmic_bytes_per_launch"] / n
        algo.setdefault("tgpu_jit_index_spec", wire)
        calls = {"decode_call": (roof["kernel"], roof["algorithmic_bytes_per_launch"] / n)}
        if "encode" in roof:
            calls["encode_call"] = (roof["encode"]["kernel"],
                                    roof["encode"]["algorithmic_bytes_per_launch"] / n)
    fetch = load(os.path.join(root, "fetch_bench"), "FETCH_SIZE")
    write = load(os.path.join(root, "write_bench"), "WRITE_SIZE")
    cfetch = load(os.path.join(root, "fetch_calib"), "FETCH_SIZE")
    cwrite = load(os.path.join(root, "write_calib"), "WRITE_SIZE")

    def avg(v):
        return sum(v) / len(v)

    ff = CALIB_BYTES / (avg(cfetch["copy_kernel"]) * 1024)
    wf = CALIB_BYTES / (avg(cwrite["copy_kernel"]) * 1024)
    res = {"config": config, "nested": nested, "records_per_launch": n,
           "wire_bytes_per_record": round(wire, 3), "record_bytes": rec,
           "source_hash": source_hash(os.path.dirname(here)),
           "commit": os.environ.get("GIT_COMMIT"),
           "calibration": {"bytes": CALIB_BYTES, "fetch_factor": round(ff, 4),
                           "write_factor": round(wf, 4)},
           "bench_value": line["value"], "bench_unit": line["unit"]}
    keep = {k for ks, _ in calls.values() for k in ks.split("+")}
    for k in sorted(set(fetch) & set(write)):
        fb = avg(fetch[k]) * 1024 * ff
        wb = avg(write[k]) * 1024 * wf
        if fb + wb < 4 * n and k not in algo and k not in keep:  # bookkeeping kernels: skip
            continue
        if k.startswith(("gen_", "elementwise", "vectorized", "unrolled", "copy")):
            continue  # data generation / torch checks, not the codec
        d = {"fetch_bytes": int(fb), "write_bytes": int(wb), "raw_fetch_kib": avg(fetch[k]),
             "raw_write_kib": avg(write[k]), "dispatches": [len(fetch[k]), len(write[k])],
             "fetch_bytes_per_record": round(fb / n, 3), "write_bytes_per_record": round(wb / n, 3),
             "hbm_bytes_per_record": round((fb + wb) / n, 3)}
        if k in algo:
            d["algorithmic_bytes_per_record"] = round(algo[k], 3)
            d["traffic_over_algorithmic"] = round((fb + wb) / n / algo[k], 4)
        res[k] = d
    for c, (ks, a) in calls.items():  # a call's kernels together vs the call's bytes
        if all(k in res for k in ks.split("+")):
            b = sum(res[k]["hbm_bytes_per_record"] for k in ks.split("+"))
            res[c] = {"kernels": ks, "hbm_bytes_per_record": round(b, 3),
                      "algorithmic_bytes_per_record": round(a, 3),
                      "traffic_over_algorithmic": round(b / a, 4)}
    with open(out_path, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


def main():
    if len(sys.argv) > 3 and sys.argv[2] == "--config":
        out = sys.argv[sys.argv.index("--out") + 1] if "--out" in sys.argv else None
        return main_config(sys.argv[1], int(sys.argv[3]), out, "--nested" in sys.argv)
    root, n = sys.argv[1], int(sys.argv[2])
    out_path = sys.argv[3] if len(sys.argv) > 3 else os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "pmc_latest.json")
    fetch = load(os.path.join(root, "fetch_bench"), "FETCH_SIZE")
    write = load(os.path.join(root, "write_bench"), "WRITE_SIZE")
    cfetch = load(os.path.join(root, "fetch_calib"), "FETCH_SIZE")
    cwrite = load(os.path.join(root, "write_calib"), "WRITE_SIZE")

    def avg(v):
        return sum(v) / len(v)

    calib = {}
    for w, k in ((16, "copy_kernel"), (8, "copy8_kernel")):
        calib[w] = {"fetch": CALIB_BYTES / (avg(cfetch[k]) * 1024),
                    "write": CALIB_BYTES / (avg(cwrite[k]) * 1024)}
    res = {"calibration": {"bytes": CALIB_BYTES,
                           "factor_by_width": {str(w): {a: round(b, 4) for a, b in c.items()}
                                               for w, c in calib.items()}},
           "records_per_launch": n}
    for k, (rw, ww) in WIDTHS.items():
        if k not in fetch or k not in write:
            continue
        fb = avg(fetch[k]) * 1024 * calib[rw]["fetch"]
        wb = avg(write[k]) * 1024 * calib[ww]["write"]
        res[k] = {"fetch_bytes": int(fb), "write_bytes": int(wb),
                  "raw_fetch_kib": avg(fetch[k]), "raw_write_kib": avg(write[k]),
                  "dispatches": [len(fetch[k]), len(write[k])],
                  "hbm_bytes_per_record": round((fb + wb) / n, 3),
                  "algorithmic_bytes_per_record": ALGO[k],
                  "traffic_over_algorithmic": round((fb + wb) / n / ALGO[k], 4)}
    with open(out_path, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
