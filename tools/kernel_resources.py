"""Summarise hipcc -Rpass-analysis=kernel-resource-usage output: one line per kernel."""
import re, subprocess, sys
src = sys.argv[1]
cmd = ['/opt/rocm/bin/hipcc', '--offload-arch=gfx950', '-O3', '-fPIC', '-std=c++17', '-Iinclude', '-c', src,
       '-o', '/tmp/_kr.o', '-Rpass-analysis=kernel-resource-usage'] + sys.argv[2:]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r'remark: (.*?): (.*?) \[', line)
    if not m:
        continue
    k, v = m.group(1).strip(), m.group(2).strip()
    if k == 'Function Name':
        cur = {'name': v}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
for r in rows:
    n = subprocess.run(['c++filt', r['name']], capture_output=True, text=True).stdout.strip()
    n = re.sub(r'\(.*', '', n)
    print(f"{n[:60]:60s} vgpr={r.get('VGPRs','?'):>4} agpr={r.get('AGPRs','?'):>3} sgpr={r.get('TotalSGPRs','?'):>4} "
          f"sspill={r.get('SGPRs Spill','?'):>4} vspill={r.get('VGPRs Spill','?'):>4} scratch={r.get('ScratchSize [bytes/lane]','?'):>4} "
          f"occ={r.get('Occupancy [waves/SIMD]','?'):>2} lds={r.get('LDS Size [bytes/block]','?')}")
