"""Summarise `hipcc -Rpass-analysis=kernel-resource-usage` output: VGPRs, spills, occupancy per kernel."""
import re
import sys

for f in sys.argv[1:]:
    cur = None
    rows = {}
    for line in open(f):
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            rows[cur] = {}
            continue
        m = re.search(r"remark:\s+(VGPRs|AGPRs|VGPRs Spill|SGPRs Spill|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\d+)", line)
        if m and cur:
            rows[cur][m.group(1)] = int(m.group(2))
    for k, v in rows.items():
        print(f"{k[:60]:60s} V={v.get('VGPRs')} A={v.get('AGPRs')} spill={v.get('VGPRs Spill')} "
              f"occ={v.get('Occupancy [waves/SIMD]')} lds={v.get('LDS Size [bytes/block]')}")
