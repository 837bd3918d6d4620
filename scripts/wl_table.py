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
