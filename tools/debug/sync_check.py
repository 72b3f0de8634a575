"""Host synchronisations inside one training step of a bench workload: torch's sync debug mode ('warn') over one
step after warm-up, each warning with the Python stack that issued it.
    python tools/debug/sync_check.py [bench.py args, e.g. --workload r3d]"""
import os
import sys
import traceback
import warnings

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.argv = [sys.argv[0], '--no-cpu-baseline'] + sys.argv[1:]
import bench  # noqa: E402


def main():
    args = bench.parse()
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(0)
    W = bench.build_workload(args, dev, 0, 1)
    for _ in range(2):
        W.step()
    torch.cuda.synchronize()
    seen = []

    def show(message, category, filename, lineno, file=None, line=None):
        seen.append((str(message), ''.join(traceback.format_stack(limit=14)[:-2])))
    warnings.showwarning = show
    torch.cuda.set_sync_debug_mode('warn')
    W.step()
    torch.cuda.set_sync_debug_mode(0)
    torch.cuda.synchronize()
    print(f'{len(seen)} synchronizing operations in one step')
    for msg, stack in seen:
        print('----', msg)
        print(stack)


if __name__ == '__main__':
    main()
