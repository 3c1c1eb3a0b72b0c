"""Static instruction census per kernel of a hipcc -S listing (device only).

  python tools/isa_census.py build/k_block.s [substring]

Counts, per kernel, the instructions by class (VALU, SALU, LDS, VMEM, SMEM,
branch/wait) and lists the most frequent VALU opcodes.  Static counts:
loops and branches are not weighted."""
import re
import sys
from collections import Counter


def kernels(text):
    for m in re.finditer(r'^(_Z\S+):\s*;', text, re.M):
        end = text.find('.Lfunc_end', m.end())
        yield m.group(1), text[m.end():end]


def klass(op):
    if op.startswith('v_'):
        return 'valu'
    if op.startswith('ds_'):
        return 'lds'
    if op.startswith(('buffer_', 'global_', 'flat_')):
        return 'vmem'
    if op.startswith(('s_load', 's_buffer_load')):
        return 'smem'
    if op.startswith(('s_waitcnt', 's_cbranch', 's_branch', 's_barrier', 's_nop', 's_setprio', 's_endpgm')):
        return 'ctl'
    if op.startswith('s_'):
        return 'salu'
    return 'other'


def main():
    text = open(sys.argv[1]).read()
    sub = sys.argv[2] if len(sys.argv) > 2 else ''
    for name, body in kernels(text):
        if sub not in name:
            continue
        ops = []
        for line in body.splitlines():
            t = line.strip()
            if not t or t.startswith(('.', ';')) or t.endswith(':'):
                continue
            ops.append(t.split()[0])
        c = Counter(klass(o) for o in ops)
        v = Counter(o for o in ops if o.startswith('v_'))
        print(name[:90])
        print('  total %d  ' % len(ops) + '  '.join('%s %d' % kv for kv in sorted(c.items())))
        print('  top VALU: ' + ', '.join('%s %d' % kv for kv in v.most_common(24)))


if __name__ == '__main__':
    main()
