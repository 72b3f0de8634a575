"""Data-parallel step of the REAL model on the GPU: two ranks (gloo, sharing the test box's
one MI355X) run `CrossModalModel` on the HIP path through `GradReducer`; the reduced gradients and the loss must
equal the single-process DataParallel equivalent (each shard through the model separately — per-replica BN — one
SigLIP loss over the global batch), reference `main.py:89-93`.

The ranks are separate processes started with subprocess from this pytest process, whose GPU probe
(`tests/conftest.py`) does not initialise HIP.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _run(tmp_path, backbone, dtype='fp32', world=2):
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK='0', WORLD_SIZE=str(world), MASTER_ADDR='127.0.0.1',
                   MASTER_PORT=str(port), CMHAR_DP_OUT=str(tmp_path), CMHAR_DP_BACKBONE=backbone,
                   CMHAR_DP_DTYPE=dtype, CMHAR_DP_BACKEND='gloo')
        procs.append(subprocess.Popen([sys.executable, '-u', os.path.join(REPO, 'tests', 'dp_worker.py')], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    logs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=100)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        logs.append(out.decode(errors='replace'))
    for p, log in zip(procs, logs):
        assert p.returncode == 0, log[-4000:]
    return [json.load(open(tmp_path / f'rank{r}.json')) for r in range(world)], \
        [json.load(open(tmp_path / f'rank{r}.sum')) for r in range(world)]


@pytest.mark.gpu
@pytest.mark.parametrize('backbone', ['videomae', 'r3d_18'])
def test_dataparallel_real_model_two_ranks(tmp_path, backbone):
    res, sums = _run(tmp_path, backbone)
    r0, r1 = res
    assert r0['sink'] == (backbone == 'videomae')
    assert r0['n_buckets'] >= 2
    # global-batch loss identical on every rank and equal to the single-process loss
    assert r0['loss'] == r1['loss']
    assert abs(r0['loss'] - r0['ref_loss']) <= 1e-6 * abs(r0['ref_loss'])
    assert r0['missing'] == []
    bad = {n: e for n, (e, norm) in r0['grad_errs'].items() if norm > 1e-6 and e > 1e-5}
    assert not bad, bad
    # same reduced gradients on both ranks (bit-identical sums)
    assert sums[0][0] == sums[0][1]
    # rank 0's BN running statistics everywhere; one checkpoint writer
    assert r0['bn_differed_before'] and r0['bn_broadcast_ok'] and r1['bn_broadcast_ok']
    assert r0['wrote_checkpoint'] and not r1['wrote_checkpoint']


@pytest.mark.gpu
def test_dataparallel_classification_global_mean(tmp_path):
    """ClassificationTrainer under GradReducer must produce the global-batch mean CE gradient."""
    res, sums = _run(tmp_path, 'classify')
    r0, r1 = res
    assert abs(r0['loss'] - r0['ref_loss']) <= 1e-5 * abs(r0['ref_loss'])
    assert abs(r1['loss'] - r0['ref_loss']) <= 1e-5 * abs(r0['ref_loss'])
    assert r0['missing'] == []
    bad = {n: e for n, (e, norm) in r0['grad_errs'].items() if norm > 1e-6 and e > 1e-5}
    assert not bad, bad
    assert sums[0][0] == sums[0][1]
