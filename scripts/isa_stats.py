#!/usr/bin/env python3
"""Instruction counts of one kernel in a hipcc --save-temps .s file.
Usage: scripts/isa_stats.py file.s 'substring of the mangled kernel name' [...]"""
import re
import sys

s = open(sys.argv[1]).read()
for pat in sys.argv[2:]:
    for m in re.finditer(r'^(_Z\S*):', s, re.M):
        name = m.group(1)
        if pat not in name:
            continue
        end = s.find('.Lfunc_end', m.end())
        lines = [l.strip() for l in s[m.end():end].splitlines()]
        lines = [l for l in lines if l and not l.startswith(('.', ';'))]
        cnt = lambda p: sum(1 for l in lines if re.search(p, l))
        print(f"{name[:90]} instr {len(lines)} dwordx4 {cnt(r'global_load_dwordx4')} dword {cnt(r'global_load_dword ')} "
              f"ushort {cnt('global_load_ushort')} scratch {cnt('scratch_')} waitcnt {cnt('s_waitcnt')} "
              f"valu {cnt(r'^v_')} salu {cnt(r'^s_(?!waitcnt|load|cbranch|branch)')} s_load {cnt(r'^s_load')} "
              f"stores {cnt(r'global_store')}")
