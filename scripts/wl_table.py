"""Table of bench.py JSON lines (gpurun_out/wl/all.jsonl): GB/s, device phase times."""
import json
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/wl/all.jsonl"
print(f"{'workload':58s} {'path':>8s} {'GB/s':>8s} {'ms/step':>8s} {'dev us':>7s} {'enc':>6s} {'sel':>6s} {'pack':>6s} "
      f"{'dec':>6s} {'encTB/s':>7s} {'hookfrac':>8s}")
for line in open(path):
    d = json.loads(line)
    p = d["phase_ms"]
    r = d["roofline"] or {}
    print(f"{d['config']['workload']:58s} {d['config'].get('hook_path', '-')[:8]:>8s} {d['value']:8.1f} {d['ms_per_step']:8.4f} "
          f"{p.get('hook_device_total', 0) * 1e3:7.1f} {p.get('encode', 0) * 1e3:6.1f} "
          f"{p.get('select', 0) * 1e3:6.1f} {p.get('pack', 0) * 1e3:6.1f} {p.get('decode', 0) * 1e3:6.1f} "
          f"{r.get('achieved', 0) / 1e3:7.2f} {r.get('hook', {}).get('frac', 0):8.3f}")
wires = []
for line in open(path):
    d = json.loads(line)
    for w in d.get("emulated_wire") or []:
        wires.append((d["config"]["workload"], d["config"].get("hook_path", "-"), w))
    fe = d.get("forced_exchange")
    if fe:
        wires.append((d["config"]["workload"], "forced", fe))
if wires:
    print()
    print("exchange path beside an emulated wire (bench line `emulated_wire`: one-rank communicator whose")
    print("all-reduce costs this GPU an R-rank ring's HBM traffic, CU footprint and time at busBW), and")
    print("forced-exchange lines (one-rank RCCL, the N > 1 code path):")
    print(f"{'workload':58s} {'line':>28s} {'per-GPU GB/s':>12s} {'x R (implied)':>13s} {'ms/bucket':>9s} "
          f"{'of wire ceiling':>15s}")
    for wl, hp, w in wires:
        if "busbw_gbs" in w:
            tag = f"emulated ws={w['emulated_ranks']} @{w['busbw_gbs']:.0f}GB/s"
            fr = w.get("frac_of_wire_ceiling")
            print(f"{wl:58s} {tag:>28s} {w['per_gpu_value']:12.1f} {w['implied_aggregate']:13.1f} {w['ms_per_bucket']:9.4f} "
                  f"{'-' if fr is None else f'{fr:.3f}':>15s}")
        else:
            print(f"{wl:58s} {'forced exchange (1-rank RCCL)':>28s} {w['value']:12.1f} {'-':>13s} {w['ms_per_bucket']:9.4f}")
