"""Per-kernel VGPRs / occupancy / LDS / scratch of one csrc file (hipcc resource-usage remarks).
Usage: python scripts/kres.py FILE REGEX"""
import re
import subprocess
import sys

f = sys.argv[1]
pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
       "-Iinclude", "-Iallreducetopk_amd/csrc", "-c", f, "-o", "/tmp/kres.o",
       "-Rpass-analysis=kernel-resource-usage"] + sys.argv[3:]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, name, d = [], None, {}
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        if name:
            rows.append((name, d))
        name, d = m.group(1), {}
        continue
    for key in ("VGPRs", "AGPRs", "Occupancy", "LDS Size", "ScratchSize"):
        m = re.search(r"\b" + re.escape(key) + r"(?: \[[^]]*\])?: (\d+)", line)
        if m:
            d[key] = m.group(1)
if name:
    rows.append((name, d))
dm = subprocess.run(["c++filt"], input="\n".join(r[0] for r in rows), capture_output=True, text=True).stdout.split("\n")
for (n, d), x in zip(rows, dm):
    x = x.replace("(anonymous namespace)::", "").replace("arctopk::", "").replace("void ", "")
    x = re.sub(r"\(.*", "", x)
    if pat.search(x):
        print(f"{x[:64]:64s} vgpr {d.get('VGPRs')} occ {d.get('Occupancy')} lds {d.get('LDS Size')} "
              f"scratch {d.get('ScratchSize')}")
