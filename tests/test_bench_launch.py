"""bench.py's launch contract: `python bench.py --gpus N` starts its N ranks itself (no external
launcher), refuses a rank count it cannot honour, and the N > 1 slab headline runs under a
watchdog.  The CPU tests run the ranks with the gloo backend and --launch-check (no GPU work);
the GPU test runs the real slab headline on one GPU with two gloo ranks."""

import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, 'bench.py')


def _run(args, env_extra=None, timeout=240):
    env = dict(os.environ)
    for k in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'LOCAL_WORLD_SIZE', 'MASTER_ADDR', 'MASTER_PORT'):
        env.pop(k, None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH] + args, cwd=REPO, env=env, capture_output=True, text=True,
                          timeout=timeout)


def _json_line(stdout):
    lines = [ln for ln in stdout.splitlines() if ln.startswith('{')]
    assert lines, stdout
    return json.loads(lines[-1])


@pytest.mark.parametrize('n', [2, 3])
def test_self_launch_gloo(n):
    """--gpus N with no WORLD_SIZE: N ranks joined one process group (all-reduce checked)."""
    p = _run(['--gpus', str(n), '--launch-check'], {'PCS_BENCH_BACKEND': 'gloo'})
    assert p.returncode == 0, p.stderr[-2000:]
    d = _json_line(p.stdout)
    assert d == {'launch_check': True, 'n_gpus': n, 'backend': 'gloo', 'parallelism': f'slab{n}',
                 'self_launched': True}


def test_gpus_exceeding_visible_devices_fails():
    """nccl needs one GPU per rank: more ranks than visible GPUs exits non-zero with a message."""
    import torch
    n = torch.cuda.device_count() + 1
    n = max(n, 2)
    p = _run(['--gpus', str(n), '--steps', '2', '--warmup', '0'])
    assert p.returncode == 2
    assert 'visible GPUs' in p.stderr


def test_world_size_mismatch_fails():
    """An external launcher whose rank count differs from --gpus is refused."""
    p = _run(['--gpus', '4', '--launch-check'], {'WORLD_SIZE': '2', 'RANK': '0', 'PCS_BENCH_BACKEND': 'gloo'})
    assert p.returncode == 2
    assert 'WORLD_SIZE=2' in p.stderr


@pytest.mark.gpu
def test_self_launch_slab_headline_gloo_one_gpu():
    """The real N = 2 slab headline on one GPU (two gloo ranks): n_gpus 2, slab2, the designed
    torch.distributed loop (no fallback)."""
    p = _run(['--gpus', '2', '--steps', '6', '--warmup', '2', '--size', '512', '--volumes', 'c4:128:f32:20', '--legs', '',
              '--no-cpu-baseline', '--headline-timeout', '100'], {'PCS_BENCH_BACKEND': 'gloo'}, timeout=110)
    assert p.returncode == 0, p.stderr[-3000:]
    d = _json_line(p.stdout)
    assert d['n_gpus'] == 2 and d['config']['parallelism'] == 'slab2'
    assert d['loop_fallback'] is False and d['value'] > 0
    # the multi-GPU lines explain themselves: compute / all-gather / exchange timed apart
    for probe in (d['comm'], d['volume_c4']['comm']):
        for k in ('compute_ms', 'allgather_ms', 'exchange_ms'):
            assert probe[k] > 0, probe
        assert probe['halo_bytes_per_side'] > 0 and probe['exchange_GBps_per_side'] > 0, probe
    v = d['volume_c4']
    assert v['steps'] == 20 and v['it_per_s'] > 0, v
    assert v['halo_bytes_per_side_per_iter'] == v['comm']['halo_bytes_per_side'], v
    # the metric as written: one --size^2 image split over the 2 ranks (strong scaling), beside the weak line
    s = d['strong_4096']
    assert s['scaling'] == 'strong' and s['it_per_s'] > 0 and s['steps'] == 6, s
    assert s['depth'] == 1 and list(s['depth_trial_ms_per_iter']) == ['1'], s  # gloo: no RCCL, depth 1 only
    assert s['comm']['exchange_ms'] > 0, s


@pytest.mark.gpu
def test_volume_leg_stall_exits_nonzero():
    """A volume leg that never returns: the watchdog prints the line with the leg's error and the
    process exits 1 (a hung first RCCL run must not read as a clean one)."""
    p = _run(['--steps', '4', '--warmup', '2', '--size', '256', '--volumes', 'c4:64:f32:2', '--legs', '',
              '--no-cpu-baseline', '--volume-timeout', '5'], {'PCS_BENCH_TEST_STALL': 'volume_c4'}, timeout=110)
    assert p.returncode == 1, (p.returncode, p.stderr[-2000:])
    d = _json_line(p.stdout)
    assert d['value'] > 0 and 'error' in d['volume_c4'], d
