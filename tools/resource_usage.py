"""Print per-kernel register / spill / occupancy for one HIP source (gfx950)."""
import re, subprocess, sys
src = sys.argv[1]
out = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-std=c++17", "-fPIC", "-c", src,
                      "-o", "/tmp/_res.o", "-Rpass-analysis=kernel-resource-usage"],
                     capture_output=True, text=True, cwd="/tmp").stderr
cur = None
rows = {}
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1); rows[cur] = {}; continue
    m = re.search(r"remark:\s+([A-Za-z \[\]/]+?):\s+(\d+)", line)
    if m and cur:
        rows[cur][m.group(1).strip()] = int(m.group(2))
for k, v in rows.items():
    if "reduce" in k or "tcsr" in k or "scan" in k: continue
    dm = subprocess.run(["c++filt", k], capture_output=True, text=True).stdout.strip()
    dm = re.sub(r"\(anonymous namespace\)::", "", dm)[:60]
    print(f"{dm:60s} V{v.get('VGPRs',0):4d} A{v.get('AGPRs',0):4d} Vsp{v.get('VGPRs Spill',0):5d} "
          f"Ssp{v.get('SGPRs Spill',0):4d} occ{v.get('Occupancy [waves/SIMD]',0)}")
