"""Per-kernel register / scratch / occupancy summary of libsparc_amp's HIP
source (hipcc -Rpass-analysis=kernel-resource-usage), filtered by a regex on
the demangled name: python scripts/kres.py 'k_secb<float, 8, 4'"""
import re
import subprocess
import sys

pat = re.compile(sys.argv[1] if len(sys.argv) > 1 else ".")
src = sys.argv[2] if len(sys.argv) > 2 else "sparc_ldpc_amd/csrc/sparc_amp.hip"
extra = sys.argv[3:]
import os
cache = "/tmp/kres_remarks.txt"
if os.environ.get("KRES_CACHED") and os.path.exists(cache):
    err = open(cache).read()
else:
    err = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                          "-Iinclude", "-fno-slp-vectorize", "-Rpass-analysis=kernel-resource-usage", "-o",
                          "/tmp/kres.so", src] + extra, capture_output=True, text=True).stderr
    open(cache, "w").write(err)
cur, rows = None, {}
for line in err.splitlines():
    m = re.search(r"remark:\s+(.*?)\s+\[-Rpass", line)
    if not m:
        continue
    txt = m.group(1)
    if txt.startswith("Function Name:"):
        cur = txt.split(":", 1)[1].strip()
        rows[cur] = {}
    elif cur and ":" in txt:
        k, v = txt.split(":", 1)
        rows[cur][k.strip()] = v.strip()
names = {}
if rows:
    dem = subprocess.run(["c++filt"], input="\n".join(rows), capture_output=True,
                         text=True).stdout.splitlines()
    names = dict(zip(rows, dem))
for k, d in rows.items():
    nm = names.get(k, k)
    if pat.search(nm):
        print(f"{nm[:90]:90s} VGPR {d.get('VGPRs', '?'):>4s} AGPR {d.get('AGPRs', '?'):>3s} "
              f"SGPR {d.get('TotalSGPRs', '?'):>4s} scratch {d.get('ScratchSize [bytes/lane]', '?'):>4s} "
              f"occ {d.get('Occupancy [waves/SIMD]', '?')}")
