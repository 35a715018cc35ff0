"""Per-kernel ISA summary from a hipcc -save-temps .s file: registers, scratch, and the compressed
instruction stream of memory / barrier / wait / MFMA ops (to check the loop's wait placement).
usage: isa_summary.py FILE.s SUBSTRING [--body]"""
import re, sys
s = open(sys.argv[1]).read()
pat = sys.argv[2]
for m in re.finditer(r'^(_Z\S*' + re.escape(pat) + r'\S*):', s, re.M):
    name = m.group(1)
    end = s.index('.Lfunc_end', m.start())
    body = s[m.start():end]
    g = lambda k: (re.search(r'\.set ' + re.escape(name) + r'\.' + k + r', (\d+)', s) or [None, '?'])[1]
    print(name, 'vgpr', g('num_vgpr'), 'agpr', g('num_agpr'), 'sgpr', g('numbered_sgpr'), 'scratch', g('private_seg_size'))
    if '--body' not in sys.argv:
        continue
    keep = ('s_waitcnt', 's_barrier', 'global_load', 'buffer_load', 'ds_read', 'ds_write', 'v_mfma', 's_setprio',
            's_cbranch', '.LBB', 's_branch', 'global_store', 'buffer_store', 'scratch_')
    comp, prev, cnt, pl = [], None, 0, ''
    for l in body.split('\n'):
        t = l.strip().split(';')[0].strip()
        if not t.startswith(keep):
            continue
        k = t.split()[0]
        if k == prev and (k.startswith(('v_mfma', 'ds_read', 'global_load_lds', 'buffer_load', 'ds_write', 'global_store', 'scratch_'))):
            cnt += 1
            continue
        if prev:
            comp.append(f'{prev} x{cnt}' if cnt > 1 else pl)
        prev, cnt, pl = k, 1, t
    comp.append(f'{prev} x{cnt}' if cnt > 1 else pl)
    print('\n'.join('   ' + c for c in comp))
