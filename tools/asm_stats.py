"""Per-function instruction statistics of a device assembly file (developer
tool): scratch ops, AGPR moves, calls, instruction count.
  hipcc ... --cuda-device-only -S -o x.s ; python tools/asm_stats.py x.s [filter]"""
import re
import sys

s = open(sys.argv[1]).read().split('\n')
pat = sys.argv[2] if len(sys.argv) > 2 else ''
cur = None
stats = {}
for l in s:
    m = re.match(r'^([_A-Za-z0-9.]+):\s*(;.*)?$', l)
    if m and not l.startswith('.L'):
        cur = m.group(1)
        stats.setdefault(cur, [0, 0, 0, 0])
    if cur is None:
        continue
    t = l.strip()
    if not t or t.startswith(('.', ';')):
        continue
    st = stats[cur]
    st[3] += 1
    if 'scratch_' in t:
        st[0] += 1
    if 'accvgpr' in t:
        st[1] += 1
    if 's_swappc' in t:
        st[2] += 1
for k, v in stats.items():
    if v[3] > 20 and pat in k:
        print(f'{k[:80]:80s} scratch {v[0]:5d} accvgpr {v[1]:5d} calls {v[2]:3d} insts {v[3]:6d}')
