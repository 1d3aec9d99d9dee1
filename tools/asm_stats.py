"""Static instruction counts of device functions in a hipcc --cuda-device-only -S listing:
python3 tools/asm_stats.py listing.s <name substring>..."""
import re
import sys
s = open(sys.argv[1]).read()
for pat in sys.argv[2:]:
    for m in re.finditer(r'^(_Z\S*' + re.escape(pat) + r'\S*):', s, re.M):
        start = m.end()
        end = s.find('.Lfunc_end', start)
        lines = [l.split(';')[0].strip() for l in s[start:end].split('\n')]
        lines = [l for l in lines if l and not l.startswith(('.', '_'))]
        ops = [l.split()[0] for l in lines]
        k = s.find('.amdhsa_kernel ' + m.group(1))
        meta = s[k:k + 4000]
        g = lambda key: (re.search(key + r'\s+(\d+)', meta) or [None, '?'])[1]
        print(f"{m.group(1)[:80]}\n  instrs {len(ops)}  v_ {sum(o.startswith('v_') for o in ops)}  s_ {sum(o.startswith('s_') for o in ops)}"
              f"  ds_ {sum(o.startswith('ds_') for o in ops)}  global_ {sum(o.startswith('global_') for o in ops)}"
              f"  vgprs {g('.amdhsa_next_free_vgpr')}  lds {g('.amdhsa_group_segment_fixed_size')}"
              f"  scratch {g('.amdhsa_private_segment_fixed_size')}")
        loads = sorted(set(o for o in ops if o.startswith('global_load')))
        print("  loads", loads)
