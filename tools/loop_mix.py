"""Instruction mix per loop of one kernel in hipcc assembly (diagnostic), from the
basic-block loop annotations ("in Loop: Header=BBx", "=>This ... Loop Header").
usage: python tools/loop_mix.py <file.s> <kernel-name-substring> [top]"""
import collections
import re
import sys


def main():
    s = open(sys.argv[1]).read()
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 12
    m = re.search(r'^(_Z\w*' + sys.argv[2] + r'\w*):', s, re.M)
    body = s[m.end():s.index('.Lfunc_end', m.end())]
    loops = collections.defaultdict(collections.Counter)
    cur = None
    for raw in body.split('\n'):
        l = raw.strip()
        if l.startswith('.LBB') or l.startswith('; %bb.'):
            lab = l.split(':')[0].lstrip('.').replace('; %bb.', 'bb.')
            mh = re.search(r'Header=(BB\d+_\d+)', l)
            if 'Loop Header' in l:
                cur = lab.replace('LBB', 'BB')
            elif mh:
                cur = mh.group(1)
            else:
                cur = None
            continue
        if not l or l.startswith((';', '.')) or cur is None:
            continue
        loops[cur][l.split()[0]] += 1
    for h, cnt in loops.items():
        n = sum(cnt.values())
        print(f"loop {h}: {n} instructions, {cnt['v_mfma_f32_16x16x32_bf16']} MFMA, "
              f"{cnt['s_waitcnt']} waitcnt, {cnt['s_and_saveexec_b64']} saveexec")
        for k, v in cnt.most_common(top):
            print(f"    {k:32s} {v}")


if __name__ == "__main__":
    main()
