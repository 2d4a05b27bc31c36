"""Does a side stream joined into a capture (wait_stream on the capturing stream) report
itself as capturing?  Dedicated (external) and pool side streams, 50 captures each."""
import os, sys, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from cloud_server_amd.utils.graphs import capture
from cloud_server_amd.utils.streams import dedicated_stream
dev = torch.device("cuda", 0)
x = torch.zeros(16, device=dev)
for kind in ("dedicated", "pool"):
    side = dedicated_stream(dev) if kind == "dedicated" else torch.cuda.Stream(dev)
    seen = []
    for i in range(50):
        g = torch.cuda.CUDAGraph()
        with capture(g):
            cur = torch.cuda.current_stream(dev)
            a = torch.cuda.is_current_stream_capturing()
            x.add_(1)
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                b = torch.cuda.is_current_stream_capturing()
                x.mul_(1)
            cur.wait_stream(side)
        seen.append((a, b))
        del g
    print(kind, "main capturing", sum(s[0] for s in seen), "side capturing", sum(s[1] for s in seen), "of", len(seen))
