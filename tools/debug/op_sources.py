"""(Used in round 3 to check which torch ops a bench step still issues — DESIGN.md §Round 3.)  Which Python call sites issue torch ops (aten::fill_ / zero_ / copy_ …) inside one bench training step:
torch.profiler CPU activity with Python stacks over one warm step of bench.py's headline workload."""
import collections
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, 'crossmodal-imu-video-ood-har_amd'))
import torch  # noqa: E402
import bench  # noqa: E402

sys.argv = ['bench.py', '--steps', '1', '--warmup', '2', '--no-cpu-baseline', '--no-trace']
args = bench.parse()
dev = torch.device('cuda', 0)
torch.cuda.set_device(0)
W = bench.build_workload(args, dev, 0, 1)
for _ in range(3):
    W.step()
torch.cuda.synchronize()
from torch.profiler import ProfilerActivity, profile  # noqa: E402
with profile(activities=[ProfilerActivity.CPU], with_stack=True, record_shapes=True) as prof:
    W.step()
    torch.cuda.synchronize()
cnt = collections.Counter()
for ev in prof.events():
    if ev.name in ('aten::fill_', 'aten::zero_', 'aten::copy_', 'aten::add_', 'aten::mul_', 'aten::cat',
                   'aten::_foreach_add_', 'aten::clone', 'aten::to', 'aten::_to_copy', 'aten::sum', 'aten::item',
                   'aten::_local_scalar_dense'):
        st = [f for f in (ev.stack or []) if 'site-packages' not in f and 'torch/' not in f][:3]
        cnt[(ev.name, str(ev.input_shapes)[:60], ' <- '.join(st))] += 1
for (name, shp, st), n in cnt.most_common(60):
    print(f'{n:4d} {name:22s} {shp:60s} {st}')
print(prof.key_averages().table(sort_by='count', row_limit=40))
