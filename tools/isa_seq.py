"""Print a kernel's instruction stream as a class string (M mfma, r/w ds_read/write, L/S vmem
load/store, B barrier, W waitcnt, X scratch, v VALU, s SALU), one line per basic block:
    python tools/isa_seq.py file.s kernel_substring [max_chars]"""
import sys


def classify(op):
    if op.startswith('v_mfma'):
        return 'M'
    if op.startswith('ds_read'):
        return 'r'
    if op.startswith('ds_write'):
        return 'w'
    if op.startswith(('buffer_load', 'global_load')):
        return 'L'
    if op.startswith(('buffer_store', 'global_store')):
        return 'S'
    if op.startswith('s_barrier'):
        return 'B'
    if op.startswith('s_waitcnt'):
        return 'W'
    if op.startswith('scratch'):
        return 'X'
    if op.startswith('v_'):
        return 'v'
    if op.startswith('s_'):
        return 's'
    return '?'


def main():
    path, sub = sys.argv[1], sys.argv[2]
    lim = int(sys.argv[3]) if len(sys.argv) > 3 else 20000
    lines = open(path).read().split('\n')
    start = next(i for i, l in enumerate(lines) if l.split(';')[0].strip().endswith(':') and sub in l and not l.startswith(('.', '\t')))
    out, cur = [], []
    for l in lines[start + 1:]:
        t = l.strip()
        if t.startswith('.Lfunc_end'):
            break
        if t.startswith('.LBB'):
            out.append(''.join(cur)); cur = [t.split(':')[0] + ': ']
            continue
        if not t or t.startswith(('.', ';')):
            continue
        cur.append(classify(t.split()[0]))
    out.append(''.join(cur))
    txt = '\n'.join(out)
    print(lines[start], 'scratch:', txt.count('X'), 'mfma:', txt.count('M'))
    print(txt[:lim])


if __name__ == '__main__':
    main()
