"""Run-length instruction sequence of one kernel in a hipcc --save-temps .s
file: python tools/isa_seq.py file.s <mangled-name-substring>"""
import sys
s = open(sys.argv[1]).read()
names = [l.split(':')[0] for l in s.splitlines() if l.startswith('_Z') and ':' in l and all(a in l.split(':')[0] for a in sys.argv[2].split(','))]
name = names[0]
i = s.index(name + ':'); j = s.index('.Lfunc_end', i)
seq = []
for l in s[i:j].splitlines():
    t = l.strip()
    if not t or t.startswith(';') or (t.startswith('.') and not t.startswith('.LBB')):
        continue
    m = t.split()[0]
    if m.startswith('v_mfma'): m = 'MFMA'
    elif m.startswith('ds_read'): m = 'DSR'
    elif m.startswith('ds_write'): m = 'DSW'
    elif m.startswith('global_load_lds'): m = 'GLDS'
    elif m.startswith('global_load'): m = 'GLD'
    elif m.startswith('s_waitcnt'): m = t.replace('s_waitcnt ', 'wait:').replace(' ', '')
    elif m.startswith('v_'): m = 'v'
    elif m.startswith('s_') and m not in ('s_barrier', 's_cbranch_scc1', 's_cbranch_scc0', 's_branch', 's_cbranch_vccnz', 's_cbranch_execz', 's_setprio'): m = 's'
    seq.append(m)
out = []; prev = None; cnt = 0
for m in seq + [None]:
    if m == prev: cnt += 1; continue
    if prev: out.append(f"{prev}x{cnt}" if cnt > 1 else prev)
    prev, cnt = m, 1
print(name); print(' '.join(out))
