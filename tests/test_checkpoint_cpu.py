"""Checkpoint interchange on the CPU (no compute): files written by the REFERENCE's trainer (fixture g9:
BaseTrainer.save_checkpoint's last.pt with optimizer + scheduler state, and a DataParallel-style `module.`-prefixed
state_dict) load into the drop-ins with strict=True via weights-only loaders; our own checkpoints round-trip."""
import json

import torch

from fixtures import fixture_config, load

GOLD = __import__('os').path.join(__import__('os').path.dirname(__file__), 'golden')


def _cfg():
    fx = load('g9_checkpoint_resume')
    return fixture_config(fx), fx


def test_reference_last_pt_loads_strict():
    from cmhar.checkpoint import load_checkpoint_file, strip_module_prefix
    from cmhar.models import CrossModalModel
    cfg, fx = _cfg()
    ckpt = load_checkpoint_file(f'{GOLD}/g9_last.pt')
    assert set(ckpt) >= {'epoch', 'model_state_dict', 'history', 'optimizer_state_dict', 'scheduler_state_dict'}
    torch.manual_seed(0)
    m = CrossModalModel(cfg)
    m.load_state_dict(strip_module_prefix(ckpt['model_state_dict']), strict=True)
    assert list(m.state_dict()) == json.loads(str(fx['keys']))


def test_module_prefixed_state_dict_is_stripped():
    from cmhar.checkpoint import load_checkpoint_file, strip_module_prefix
    from cmhar.models import CrossModalModel
    cfg, _ = _cfg()
    ckpt = load_checkpoint_file(f'{GOLD}/g9_module_prefixed.pt')
    assert all(k.startswith('module.') for k in ckpt['model_state_dict'])
    m = CrossModalModel(cfg)
    m.load_state_dict(strip_module_prefix(ckpt['model_state_dict']), strict=True)


def test_optimizer_state_maps_onto_same_parameter_order():
    """torch's Optimizer.load_state_dict maps state by parameter position: the drop-in must register parameters
    in the reference's order (shapes line up one to one)."""
    from cmhar.checkpoint import load_checkpoint_file
    from cmhar.models import CrossModalModel
    cfg, _ = _cfg()
    ckpt = load_checkpoint_file(f'{GOLD}/g9_last.pt')
    m = CrossModalModel(cfg)
    params = list(m.parameters())
    st = ckpt['optimizer_state_dict']['state']
    assert len(ckpt['optimizer_state_dict']['param_groups'][0]['params']) == len(params)
    for i, p in enumerate(params):
        if i in st:
            assert tuple(st[i]['exp_avg'].shape) == tuple(p.shape), i


def test_own_checkpoint_round_trip(tmp_path):
    from cmhar.checkpoint import load_checkpoint_file, save_final_state_dict
    from cmhar.models import CrossModalModel
    cfg, _ = _cfg()
    torch.manual_seed(1)
    m = CrossModalModel(cfg)
    p = save_final_state_dict(m, tmp_path / 'cross_modal' / 'final_model_state_dict.pt')
    sd = load_checkpoint_file(p)
    m2 = CrossModalModel(cfg)
    m2.load_state_dict(sd, strict=True)
    for (k, a), (_, b) in zip(m.state_dict().items(), m2.state_dict().items()):
        assert torch.equal(a, b), k
