"""Summarise rocprofv3 --pmc CSVs (tools/pmc.sh) per gsr kernel: counter means per
dispatch, derived HBM bytes (gfx950: FETCH_SIZE reads half of a wide streaming
read -> doubled, per MI355X_MICROARCH.md §HBM; WRITE_SIZE as is), and write
profiles/pmc_summary.json for bench.py's roofline `traffic` field."""
import csv
import glob
import json
import sys
from collections import defaultdict
from pathlib import Path

d = Path(sys.argv[1])
out = Path(sys.argv[2]) if len(sys.argv) > 2 else None
SUFFIX = sys.argv[3] if len(sys.argv) > 3 else ""  # e.g. "_E" for a config E pass
vals = defaultdict(lambda: defaultdict(list))
dur = defaultdict(list)
for f in sorted(glob.glob(str(d / "**" / "*counter_collection.csv"), recursive=True)):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
STAGE = {"gsr::preprocess_fwd_kernel": "preprocess", "gsr::render_fwd_kernel": "render_fwd",
         "gsr::render_bwd_kernel": "render_bwd", "gsr::preprocess_bwd_kernel": "preprocess_bwd",
         "gsr::emit_kernel": "duplicate", "gsr::bwd_prepare_kernel": "bwd_prepare"}
summary = {"note": "per-dispatch means; hbm_bytes = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 FETCH_SIZE "
                   "counts half of wide streaming reads, MI355X_MICROARCH.md §HBM)", "kernels": {}, "stages": {}}
for k, cs in sorted(vals.items()):
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    line = {c: round(x, 1) for c, x in m.items()}
    if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
        hbm = 2 * m["FETCH_SIZE"] * 1024 + m["WRITE_SIZE"] * 1024
        line["hbm_bytes_per_launch"] = hbm
        line["dispatches"] = len(cs["FETCH_SIZE"])
        for kn, st in STAGE.items():
            if k.startswith(kn):
                summary["stages"][st + SUFFIX] = {"hbm_bytes_per_launch": hbm, "kernel": k}
    if "SQ_WAVE_CYCLES" in m and "SQ_WAVES" in m and m["SQ_WAVES"]:
        line["cycles_per_wave"] = round(m["SQ_WAVE_CYCLES"] / m["SQ_WAVES"], 1)
    if "SQ_INSTS_VALU" in m and "SQ_WAVES" in m and m["SQ_WAVES"]:
        line["valu_per_wave"] = round(m["SQ_INSTS_VALU"] / m["SQ_WAVES"], 1)
    if "SQ_INSTS_VALU" in m and m.get("GRBM_GUI_ACTIVE"):
        # VALU issue utilisation: a wave64 f32 VALU op holds a SIMD 2 cycles when two
        # waves interleave (MI355X_MICROARCH.md cycle constants); 1024 SIMDs; the
        # kernel's cycles = GRBM_GUI_ACTIVE / 8 (summed over the 8 XCDs)
        line["valu_issue_frac"] = round(2.0 * m["SQ_INSTS_VALU"] / (1024 * m["GRBM_GUI_ACTIVE"] / 8), 3)
    summary["kernels"][k] = line
    print(k)
    for c, x in sorted(line.items()):
        print(f"    {c:28s} {x:>16,.1f}" if isinstance(x, float) else f"    {c:28s} {x}")
# multi-kernel stages: HBM bytes of one stage launch = per-dispatch means times the
# dispatches of each kernel per launch.  The radix kernels serve both sorts; their
# template arguments tell them apart (gsr_common.hpp tsort_items/dsort_items: tile
# sort <8, mode> at config C, <16, mode> at E; depth sort <4, 0> at C, <8, 0> at
# E; mode 1 / 2 = the packed two-pass tile sort, 0 = plain key/value passes).
# radix_digit_scan_kernel is shared and small (256 x blocks counters): its mean is
# counted once per pass.
def tile_sort_stage(kernels, titems, suffix=""):
    """One tile-sort launch: the packed two passes (binning.hip) when their
    kernels were traced, else the plain passes + identify_ranges."""
    def mean(prefix):
        for k, line in kernels.items():
            if k.startswith(prefix) and k.endswith(suffix) and (suffix or not k.endswith("_E")) \
                    and "hbm_bytes_per_launch" in line:
                return line["hbm_bytes_per_launch"]
        return None
    up, down = "gsr::radix_upsweep_kernel", "gsr::radix_downsweep_kernel"
    packed = [(f"{up}<{titems}, 1>", 1), (f"{down}<{titems}, 1>", 1), (f"{up}<{titems}, 2>", 1),
              (f"{down}<{titems}, 2>", 1), ("gsr::radix_digit_scan_kernel", 2)]
    plain = [(f"{up}<{titems}, 0>", 2), (f"{down}<{titems}, 0>", 2), ("gsr::radix_digit_scan_kernel", 2),
             ("gsr::identify_ranges_kernel", 1)]
    for parts in (packed, plain):
        got = [(mean(k), n) for k, n in parts]
        if all(v is not None for v, _ in got):
            return {"hbm_bytes_per_launch": sum(v * n for v, n in got),
                    "kernel": " + ".join(f"{n} x {k}" for k, n in parts)}
    return None


rec = tile_sort_stage(summary["kernels"], "16" if SUFFIX.startswith("_E") else "8")
if rec:
    summary["stages"]["tile_sort" + SUFFIX] = rec


def rowspan_stages(kernels):
    """The row-span binning (rowspan.hip): duplicate = pass A; tile_sort = pass B's
    counts + one digit scan + its scatter; scan = the rank gather + one digit scan."""
    def find(prefix):
        for k, line in kernels.items():
            if k.startswith(prefix) and "hbm_bytes_per_launch" in line:
                return k, line["hbm_bytes_per_launch"]
        return None, None
    out = {}
    ka, a = find("gsr::rowspan_a_kernel")
    kc, c = find("gsr::rowspan_b_count_kernel")
    kb, b = find("gsr::rowspan_b_kernel")
    ks, sc = find("gsr::radix_digit_scan_kernel")
    kg, g = find("gsr::rank_gather_kernel")
    if a is not None:
        out["duplicate"] = {"hbm_bytes_per_launch": a, "kernel": ka}
    if None not in (c, b, sc):
        out["tile_sort"] = {"hbm_bytes_per_launch": c + sc + b, "kernel": f"{kc} + {ks} + {kb}"}
    if None not in (g, sc):
        out["scan"] = {"hbm_bytes_per_launch": g + sc, "kernel": f"{kg} + {ks}"}
    return out


for st, rec in rowspan_stages(summary["kernels"]).items():
    summary["stages"][st + SUFFIX] = rec
# One benchmark unit's measured HBM bytes (bench.py iter_hbm_frac_measured): every
# gsr kernel's per-dispatch bytes times its dispatches, over the units the run made.
# The run repeats one unit (tools/pmc.sh: warm-up, stage split and timed steps of
# the same step; bench.py reads num_rendered from the warm-up, no extra forward), so
# the anchor kernel — once per unit: render_bwd for a training step, render_fwd for
# a forward-only config — counts the units.
ks = {k: v for k, v in summary["kernels"].items() if "dispatches" in v}
anchor = next((k for k in ks if k.startswith("gsr::render_bwd_kernel")), None) or \
    next((k for k in ks if k.startswith("gsr::render_fwd_kernel")), None)
if anchor:
    units = ks[anchor]["dispatches"]
    total = sum(v["hbm_bytes_per_launch"] * v["dispatches"] for v in ks.values())
    summary["units"] = {"unit" + SUFFIX: {"hbm_bytes_per_unit": total / units, "units": units, "anchor": anchor,
                                          "kernels": sorted(ks)}}
for st, rec in summary["stages"].items():
    frac = summary["kernels"].get(rec["kernel"], {}).get("valu_issue_frac")
    if frac is not None:
        rec["valu_issue_frac"] = frac
if out:
    if out.exists() and "--merge" in sys.argv:  # keep the other config's stages
        old = json.loads(out.read_text())
        old.get("stages", {}).update(summary["stages"])
        old.setdefault("units", {}).update(summary.get("units", {}))
        old.get("kernels", {}).update({k + SUFFIX: v for k, v in summary["kernels"].items()})
        summary = old
    out.write_text(json.dumps(summary, indent=1) + "\n")
