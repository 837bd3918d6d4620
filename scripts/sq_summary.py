"""Per-kernel SQ counter summary of rocprofv3 --pmc passes (scripts/gpu_r4counters.sh).

    python scripts/sq_summary.py DIR [KERNEL_SUBSTR ...]

For each kernel (averaged over its dispatches): duration, waves, VGPRs, instructions per wave
(VALU / SALU / VMEM read / VMEM write / LDS / SMEM), and where the wave cycles go
(SQ_WAVE_CYCLES = ACTIVE_INST_ANY + WAIT_INST_ANY + WAIT_ANY, quad-cycles: MI355X_MICROARCH.md
rocprofv3 PMC section): the share of wave time spent issuing, stalled at issue, or parked on
s_waitcnt / barriers -- latency-bound kernels park, issue-bound kernels issue.  Also the
average waves resident per CU (WAVE_CYCLES / BUSY_CYCLES over the CUs' share), and the
effective clock (GRBM_GUI_ACTIVE / 8 XCDs / duration)."""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1]
want = sys.argv[2:]
acc = defaultdict(lambda: defaultdict(list))
meta = {}
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    with open(f) as fh:
        for r in csv.DictReader(fh):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").strip()
            k = k.split("<")[0] + ("<" + k.split("<", 1)[1] if "<" in k else "")
            if want and not any(w in k for w in want):
                continue
            did = (f, r["Dispatch_Id"])
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            acc[k]["_dur_" + os.path.basename(os.path.dirname(f))].append(dur)
            meta[k] = (int(r["Grid_Size"]), int(r["Workgroup_Size"]), int(r["VGPR_Count"]),
                       int(r["Accum_VGPR_Count"]), int(r["LDS_Block_Size"]))


def avg(d, n):
    v = d.get(n)
    return sum(v) / len(v) if v else float("nan")


print(f"{'kernel':44s} {'us':>7s} {'waves':>7s} {'vgpr':>4s} {'lds':>6s} | per wave: {'valu':>6s} {'salu':>5s} "
      f"{'vmrd':>5s} {'vmwr':>5s} {'lds':>5s} {'smem':>5s} | cyc/wave {'active':>6s} {'instst':>6s} {'park':>6s}"
      f" | waves/CU {'GHz':>5s}")
for k in sorted(acc, key=lambda k: -avg(acc[k], "SQ_WAVE_CYCLES")):
    d = acc[k]
    w = avg(d, "SQ_WAVES")
    if not w or w != w:
        continue
    durs = [v for n, v in d.items() if n.startswith("_dur_")]
    dur = sum(sum(v) / len(v) for v in durs) / len(durs)
    pw = lambda n: avg(d, n) / w  # noqa: E731
    wc = avg(d, "SQ_WAVE_CYCLES")
    act, ist, park = (avg(d, n) / wc if wc else float("nan") for n in
                      ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY"))
    busy = avg(d, "SQ_BUSY_CYCLES")
    ghz = avg(d, "GRBM_GUI_ACTIVE") / 8 / (dur * 1e3) if dur else float("nan")
    # waves resident per CU: wave-cycles (quad-cycles, x4 = cycles) over the kernel's cycles x 256 CUs
    wpc = 4 * wc / (dur * 1e3 * ghz * 256) if dur and ghz == ghz else float("nan")
    g, wg, vg, ag, lds = meta[k]
    print(f"{k[:44]:44s} {dur:7.1f} {w:7.0f} {vg + ag:4d} {lds:6d} | {pw('SQ_INSTS_VALU'):16.0f} "
          f"{pw('SQ_INSTS_SALU'):5.0f} {pw('SQ_INSTS_VMEM_RD'):5.1f} {pw('SQ_INSTS_VMEM_WR'):5.1f} "
          f"{pw('SQ_INSTS_LDS'):5.1f} {pw('SQ_INSTS_SMEM'):5.1f} | {wc / w * 4:8.0f} {act:6.2f} {ist:6.2f} "
          f"{park:6.2f} | {wpc:8.1f} {ghz:5.2f}")
