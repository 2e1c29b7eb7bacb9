"""Static check of the LDS-DMA waits (round 5; every DMA site since round 6).

Every kernel of an assembly file (hipcc -S) that issues `buffer_load ... lds` is scanned site by
site: the DMA loads between two `s_waitcnt vmcnt` are one group, and the first `s_barrier` after the
group that follows a vmcnt wait is the one that publishes the group's LDS tile.  Before that barrier
some `s_waitcnt vmcnt(N)` must see at least N vector-memory loads issued after the group's last DMA
load; otherwise a DMA load may still be in flight when the tile is read.  A kernel whose loop the
compiler inlined several times (peeled prologue, interior-only loop, mixed loop) has one group per
copy, and each is checked -- a single-site check (the round-5 form) only saw the textually last one."""
import re
import sys

_WAIT = re.compile(r's_waitcnt\b.*\bvmcnt\((\d+)\)')


def _is_dma(l):
    return l.startswith('buffer_load') and l.endswith(' lds')


def _is_vmem_load(l):
    return (l.startswith('buffer_load') or l.startswith('global_load')) and not l.endswith(' lds')


def check_body(body):
    """[(site index, ok, wait N, loads after the group)] for every DMA group of one kernel body."""
    out = []
    i, n = 0, len(body)
    while i < n:
        if not _is_dma(body[i]):
            i += 1
            continue
        # the group: DMA loads until the next vmcnt wait (other instructions may sit between them)
        last, j = i, i + 1
        while j < n and not _WAIT.search(body[j]) and not body[j].startswith('s_barrier'):
            if _is_dma(body[j]):
                last = j
            j += 1
        n_after, waits, verdict = 0, [], None
        for l in body[last + 1:]:
            if _is_vmem_load(l):
                n_after += 1
            m = _WAIT.search(l)
            if m:
                waits.append((int(m.group(1)), n_after))
            if l.startswith('s_barrier') and waits:
                ok = any(w <= a for w, a in waits)
                verdict = (ok, min(w for w, _ in waits), n_after)
                break
        if verdict is None:
            verdict = (False, None, n_after)
        out.append((last,) + verdict)
        i = last + 1
    return out


def check(path, pattern=r'^_Z\w+:'):
    lines = open(path).read().split('\n')
    starts = [i for i, l in enumerate(lines) if re.match(pattern, l)]
    bad = 0
    for s in starts:
        name = lines[s].split(':')[0]
        e = s + 1
        while e < len(lines) and not lines[e].startswith('.Lfunc_end'):
            e += 1
        body = [l.strip() for l in lines[s:e]]
        sites = check_body(body)
        if not sites:
            continue
        nbad = sum(not ok for _, ok, _, _ in sites)
        bad += nbad
        detail = ' '.join(f'[{w}<={a}]' if ok else f'[RACE {w}>{a}]' for _, ok, w, a in sites)
        print(('ok  ' if not nbad else 'RACE'), name[:70], f'{len(sites)} DMA sites', detail)
    return bad


if __name__ == '__main__':
    sys.exit(1 if sum(check(p) for p in sys.argv[1:]) else 0)
