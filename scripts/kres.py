"""kernel resource usage from hipcc -Rpass-analysis=kernel-resource-usage output: name VGPRs scratch LDS"""
import re, subprocess, sys
src = sys.argv[1]
flags = "-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-fast-math".split()
extra = sys.argv[2:]
p = subprocess.run(["/opt/rocm/bin/hipcc", *flags, *extra, "-c", src, "-o", "/tmp/kres.o",
                    "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True)
cur = None
rows = {}
for line in p.stderr.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1); rows[cur] = {}
        continue
    for k in ["VGPRs", "ScratchSize \\[bytes/lane\\]", "LDS Size \\[bytes/block\\]", "Occupancy \\[waves/SIMD\\]"]:
        m = re.search(k + r": (\d+)", line)
        if m and cur:
            rows[cur][k.split()[0]] = int(m.group(1))
for k, v in sorted(rows.items()):
    print(f"{v.get('VGPRs')}\t{v.get('ScratchSize')}\t{v.get('Occupancy')}\t{v.get('LDS')}\t{k[:110]}")
