"""Per-kernel instruction census of a hipcc -S listing (development aid)."""
import re
import sys

F64 = re.compile(r'v_\w+_f64')
s = open(sys.argv[1]).read()
heads = [(m.start(), m.group(1)) for m in re.finditer(r'^(_Z\S+):\s*;\s*@', s, re.M)]
for pos, name in heads:
    end = s.find('.Lfunc_end', pos)
    body = s[pos:end]
    ins = [l.split()[0] for l in body.splitlines() if l.startswith('\t') and l.strip() and not l.strip().startswith(('.', ';'))]
    valu = sum(1 for i in ins if i.startswith('v_'))
    nf64 = len(F64.findall(body))
    print(f"{name[:60]:60s} instr {len(ins):6d} valu {valu:5d} sad {body.count('v_sad_u8'):4d} "
          f"align {body.count('v_alignbyte'):4d} ds_read {body.count('ds_read'):4d} "
          f"ds_write {body.count('ds_write'):3d} bperm {body.count('ds_bpermute'):3d} "
          f"readlane {body.count('v_readlane'):3d} writelane {body.count('v_writelane'):3d} "
          f"scratch {body.count('scratch_'):3d} f64 {nf64:3d}")
