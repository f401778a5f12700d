"""Static instruction mix of one kernel in a hipcc --save-temps .s file.
usage: python tools/isa_stats.py <file.s> <mangled-name-substring> [--dump out.s]"""
import collections, re, sys

def body_of(path, key):
    s = open(path).read()
    m = re.search(r'^(\S*%s\S*):\s*;' % re.escape(key), s, re.M)
    i = m.start()
    j = s.index('.Lfunc_end', i)
    return s[i:j]

def classify(m):
    if m.startswith('v_mfma'): return 'mfma'
    if m.startswith(('v_readlane', 'v_writelane', 'v_readfirstlane')): return 'lane'
    if m.startswith('v_pk_'): return 'valu_pk'
    if m.startswith('v_'): return 'valu'
    if m.startswith('s_waitcnt'): return 'wait'
    if m.startswith('s_'): return 'salu'
    if m.startswith('ds_'): return 'lds'
    if m.startswith(('buffer', 'global', 'flat', 'scratch')): return 'vmem'
    return m

if __name__ == '__main__':
    body = body_of(sys.argv[1], sys.argv[2])
    if '--dump' in sys.argv:
        open(sys.argv[sys.argv.index('--dump') + 1], 'w').write(body)
    ins = [l.split()[0] for l in (x.strip() for x in body.split('\n'))
           if l and not l.startswith(('.', ';')) and not l.endswith(':')]
    c = collections.Counter(ins)
    cls = collections.Counter()
    for m, n in c.items(): cls[classify(m)] += n
    print(len(ins), dict(cls))
    for m, n in c.most_common(45): print('%6d %s' % (n, m))
