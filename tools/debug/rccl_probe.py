"""Can two ranks share the one GPU of a test box over RCCL (backend "nccl")?  Spawns 2 processes on cuda:0, each
all-reduces a tensor; prints the result or the error.  python tools/debug/rccl_probe.py [world]"""
import os
import socket
import subprocess
import sys

if os.environ.get('PROBE_RANK') is None:
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    procs = [subprocess.Popen([sys.executable, __file__], env=dict(os.environ, PROBE_RANK=str(r), WORLD_SIZE=str(world),
                              MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))) for r in range(world)]
    rc = [p.wait(timeout=120) for p in procs]
    print('exit codes', rc)
    sys.exit(max(rc))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
r = int(os.environ['PROBE_RANK'])
w = int(os.environ['WORLD_SIZE'])
torch.cuda.set_device(0)
dist.init_process_group('nccl', rank=r, world_size=w, device_id=torch.device('cuda', 0))
t = torch.full((1 << 20,), float(r + 1), device='cuda')
dist.all_reduce(t)
torch.cuda.synchronize()
print(f'rank {r}: all_reduce -> {t[0].item()} (expected {w * (w + 1) / 2})', flush=True)
dist.destroy_process_group()
