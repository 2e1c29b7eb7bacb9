"""Static check of the row-march kernels' LDS-DMA waits (round 5): in the main loop of every
k_pds2d_nmarch* kernel of an assembly file (hipcc -S), the `s_waitcnt vmcnt(N)` before the barrier that
precedes the first read of the z tiles must see at least N plain loads issued after the step's last
`buffer_load ... lds`; otherwise a DMA load may still be in flight when the tile is read."""
import re
import sys


def check(path):
    lines = open(path).read().split('\n')
    starts = [i for i, l in enumerate(lines) if re.match(r'^_ZN3pcs\w*k_pds2d_nmarch\w*:', l)]
    bad = 0
    for s in starts:
        name = lines[s].split(':')[0]
        e = s + 1
        while not lines[e].startswith('.Lfunc_end'):
            e += 1
        body = [l.strip() for l in lines[s:e]]
        dma = [i for i, l in enumerate(body) if l.startswith('buffer_load') and l.endswith(' lds')]
        if not dma:
            continue
        last = dma[-1]
        n_after, verdict = 0, None
        for l in body[last + 1:]:
            if l.startswith('buffer_load') and not l.endswith(' lds'):
                n_after += 1
            m = re.match(r's_waitcnt vmcnt\((\d+)\)', l)
            if m:
                n = int(m.group(1))
                verdict = (n, n_after)
            if l.startswith('s_barrier') and verdict is not None:
                break
        ok = verdict is not None and verdict[1] >= verdict[0]
        bad += not ok
        print(('ok  ' if ok else 'RACE'), name[:70], 'wait vmcnt', verdict[0] if verdict else None, 'loads after DMA', n_after)
    return bad


if __name__ == '__main__':
    sys.exit(1 if sum(check(p) for p in sys.argv[1:]) else 0)
