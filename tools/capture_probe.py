"""Root-cause probe for GPUTEST_r04's capture failure: does pnr_destroy (hipFree /
hipHostFree / hipEventDestroy of a built grid) inside a global-mode torch graph
capture invalidate it?  Prints one line per case; never used by the product."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from pointnerf_amd import _lib as L  # noqa: E402
from pointnerf_amd.querier import GridHandle  # noqa: E402
from scenes import scene  # noqa: E402


def case(mode):
    dev = torch.device("cuda:0")
    sc = scene(20000, H=8, W=8)
    h = GridHandle(dev)
    h.build(sc["opt"], torch.from_numpy(sc["xyz"]).to(dev).contiguous())
    torch.cuda.synchronize()
    raw = h.h
    h.h = None
    x = torch.zeros(4, device=dev)
    g = torch.cuda.CUDAGraph()
    try:
        with torch.cuda.graph(g, capture_error_mode=mode):
            L.lib().pnr_destroy(raw)       # what GridHandle.__del__ did in round 4
            x.add_(1.0)
        print(f"{mode}: capture valid after pnr_destroy inside it")
    except Exception as e:  # noqa: BLE001
        print(f"{mode}: capture INVALIDATED: {str(e).splitlines()[0]}")
    torch.cuda.synchronize()


if __name__ == "__main__":
    # one mode per process: an invalidated capture leaves the stream unusable
    case(sys.argv[1] if len(sys.argv) > 1 else "global")
