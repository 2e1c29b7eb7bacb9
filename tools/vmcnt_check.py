"""Static check of the LDS-DMA waits (round 5; every DMA site since round 6).

Every kernel of an assembly file (hipcc -S) that issues `buffer_load ... lds` is scanned site by
site: the DMA loads between two `s_waitcnt vmcnt` are one group, and the first `s_barrier` after the
group that follows a vmcnt wait is the one that publishes the group's LDS tile.  Before that barrier
some `s_waitcnt vmcnt(N)` must see at least N vector-memory loads issued after the group's last DMA
load; otherwise a DMA load may still be in flight when the tile is read.  A kernel whose loop the
compiler inlined several times (peeled prologue, interior-only loop, mixed loop) has one group per
copy, and each is checked -- a single-site check (the round-5 form) only saw the textually last one.
check() follows every path of the control-flow graph from each DMA load (check_body_cfg): a loop the
compiler lays out of line is read as it runs, not as it is printed."""
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


_LABEL = re.compile(r'^(\.?[A-Za-z_][\w.$]*):')
_BRANCH = re.compile(r'^s_(c?branch)\w*\s+(\S+)')


def check_body_cfg(body):
    """check_body over the control-flow graph: every DMA load is followed along every path (branch
    targets and fall-throughs) to the first s_barrier; some `s_waitcnt vmcnt(N)` on the path must see at
    least N vector-memory loads issued after that DMA load.  A path that meets another DMA load first is
    that load's to check (vmcnt retires in order).  The compiler may lay a loop out of line (a DMA loop
    placed after the code it exits to), which the linear scan of check_body misreads.
    [(site index, ok, min wait N seen, loads on the failing path or the min over paths)]"""
    labels = {}
    for i, l in enumerate(body):
        m = _LABEL.match(l)
        if m:
            labels[m.group(1)] = i
    out = []
    for d, l in enumerate(body):
        if not _is_dma(l):
            continue
        ok, waits, worst = True, [], None
        seen = set()
        stack = [(d + 1, 0)]
        while stack:
            i, n = stack.pop()
            done = False
            while i < len(body):
                if (i, n) in seen:
                    done = True
                    break
                seen.add((i, n))
                ins = body[i]
                if _is_dma(ins):
                    done = True
                    break
                if _is_vmem_load(ins):
                    n = min(n + 1, 63)
                m = _WAIT.search(ins)
                if m:
                    w = int(m.group(1))
                    waits.append(w)
                    if w <= n:
                        done = True
                        break
                if ins.startswith('s_barrier'):
                    ok, worst = False, n if worst is None else min(worst, n)
                    done = True
                    break
                if ins.startswith('s_endpgm'):
                    done = True
                    break
                b = _BRANCH.match(ins)
                if b:
                    tgt = labels.get(b.group(2))
                    if tgt is not None:
                        stack.append((tgt + 1, n))
                    if b.group(1) == 'branch':  # unconditional: no fall-through
                        done = True
                        break
                i += 1
            if not done:
                continue
        out.append((d, ok, min(waits) if waits else None, worst if worst is not None else 0))
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
        sites = check_body_cfg(body)
        if not sites:
            continue
        nbad = sum(not ok for _, ok, _, _ in sites)
        bad += nbad
        detail = ' '.join('[ok]' if ok else f'[RACE wait {w} > {a} loads]' for _, ok, w, a in sites)
        print(('ok  ' if not nbad else 'RACE'), name[:70], f'{len(sites)} DMA sites', detail)
    return bad


if __name__ == '__main__':
    sys.exit(1 if sum(check(p) for p in sys.argv[1:]) else 0)
