#!/usr/bin/env python3
"""isa_count.py -- static instruction counts per kernel of a hipcc -save-temps .s file.

Usage: isa_count.py <file.s> [kernel-substring ...]

For every kernel symbol (optionally only those containing one of the substrings) prints the
VALU total and the counts of the instruction kinds the bit-sliced kernels are made of, plus the
VGPR / spill figures of the kernel descriptor.  Used to check that a probe variant still
contains the work it claims to time (variants whose math the compiler deleted).
"""
import collections
import re
import sys

KINDS = ['v_bitop3_b32', 'v_perm_b32', 'v_lshlrev_b32', 'v_lshrrev_b32', 'v_xor_b32', 'v_mov_b32_dpp',
         'ds_read_b128', 'ds_read_b64', 'ds_write_b128', 'ds_write_b64', 'global_load_lds_dwordx4',
         'buffer_load_dwordx4', 'global_store_dwordx4', 'global_store_dwordx2', 'scratch_load_dword',
         'scratch_load_dwordx2', 'scratch_store_dword', 'scratch_store_dwordx2', 's_barrier', 's_waitcnt']


def kernels(text):
    out = {}
    for m in re.finditer(r'^(_Z\w+):\s*;\s*@', text, re.M):
        name = m.group(1)
        end = text.find('.Lfunc_end', m.end())
        out[name] = text[m.end():end]
    return out


def meta(text, name):
    """VGPRs and scratch from the kernel descriptor (.amdhsa_kernel block)."""
    m = re.search(r'\.amdhsa_kernel\s+' + re.escape(name) + r'\s*\n', text)
    res = {}
    if not m:
        return res
    blk = text[m.end():text.find('.end_amdhsa_kernel', m.end())]
    for key, lab in (('next_free_vgpr', 'vgpr'), ('private_segment_fixed_size', 'scratch_bytes'),
                     ('next_free_sgpr', 'sgpr')):
        mm = re.search(r'\.amdhsa_' + key + r'\s+(\d+)', blk)
        if mm:
            res[lab] = int(mm.group(1))
    return res


def count(body):
    c = collections.Counter()
    for line in body.split('\n'):
        t = line.strip().split()
        if not t or t[0].startswith(('.', ';')) or t[0].endswith(':'):
            continue
        c[t[0]] += 1
    return c


def main():
    text = open(sys.argv[1]).read()
    subs = sys.argv[2:]
    for name, body in kernels(text).items():
        if subs and not any(s in name for s in subs):
            continue
        c = count(body)
        valu = sum(v for k, v in c.items() if k.startswith('v_'))
        kinds = ' '.join(f'{k}={c[k]}' for k in KINDS if c[k])
        print(f'{name}: VALU {valu} {kinds} {meta(text, name)}')


if __name__ == '__main__':
    main()
