"""Instruction histogram of the MFMA main loop of each kernel in a device .s file.
python tools/loop_hist.py FILE.s REGEX"""
import collections
import re
import sys

s = open(sys.argv[1]).read()
pat = re.compile(sys.argv[2])
for name in re.findall(r'^(_Z[^\s:]+):', s, re.M):
    if not pat.search(name):
        continue
    body = s[s.index('\n' + name + ':') + 1:]
    body = body[:body.index('.Lfunc_end')].split('\n')
    labels = {l.split(':')[0]: i for i, l in enumerate(body) if re.match(r'^\.LBB\S+:', l)}
    best = None
    for i, l in enumerate(body):
        m = re.match(r'^\s+s_(cbranch_\w+|branch)\s+(\.LBB\S+)', l)
        if m and m.group(2) in labels and labels[m.group(2)] < i:
            seg = body[labels[m.group(2)]:i + 1]
            if any('mfma' in x for x in seg) and (best is None or len(seg) > len(best)):
                best = seg
    if not best:
        continue
    ins = [l.split()[0] for l in best if l.startswith('\t') and not l.startswith(('\t.', '\t;'))]
    c = collections.Counter(ins)
    grp = collections.Counter()
    for k, n in c.items():
        g = 'mfma' if 'mfma' in k else k.split('_')[0] + ('_' + k.split('_')[1] if k.startswith(('ds', 'global', 'buffer')) else '')
        grp[g] += n
    print(name, len(ins), dict(grp))
    if len(sys.argv) > 3:
        print('  ', c.most_common(int(sys.argv[3])))
