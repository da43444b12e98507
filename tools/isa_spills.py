#!/usr/bin/env python3
"""Where a kernel's scratch spills sit: for one kernel of a --save-temps .s
file, print the line of every scratch load/store with the loop depth of the
basic block it is in (LLVM's '; %bb... Loop Depth N' comments).
    python tools/isa_spills.py FILE.s MANGLED-SUBSTRING"""
import re
import sys

s = open(sys.argv[1]).read()
key = sys.argv[2]
names = [m for m in re.findall(r'^(\S+):\s*;\s*@', s, re.M) if key in m and m.startswith('_Z')]
name = names[0]
a = s.index(name + ':')
b = s.index('.Lfunc_end', a)
body = s[a:b].split('\n')
depth = 0
n = {}
for i, l in enumerate(body):
    m = re.search(r'Loop Depth=(\d+)', l)
    if re.match(r'^\.LBB', l):
        depth = int(m.group(1)) if m else 0
    if 'scratch_' in l or ('buffer_' in l and 'off, s[0:3]' in l):
        n[depth] = n.get(depth, 0) + 1
        if len(sys.argv) > 3:
            print(i, depth, l.strip())
print(name[:90], "instructions", len(body), "scratch ops by loop depth", n)
