"""Which threads does a world-1 RCCL process group start, with and without
TORCH_NCCL_BLOCKING_WAIT, and does the watchdog query eager works' events?
Prints one JSON line per mode (run as a child per mode: the env is read at PG creation)."""
import json
import os
import sys


def threads():
    out = []
    for t in sorted(os.listdir("/proc/self/task")):
        try:
            with open(f"/proc/self/task/{t}/comm") as f:
                out.append(f.read().strip())
        except OSError:
            pass
    return out


def child():
    import socket
    import time
    import torch
    import torch.distributed as dist
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    before = threads()
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    t = torch.ones(16, device="cuda")
    dist.all_reduce(t)
    torch.cuda.synchronize()
    time.sleep(0.5)
    after = threads()
    new = sorted(set(after) - set(before))
    print(json.dumps({"blocking_wait": os.environ.get("TORCH_NCCL_BLOCKING_WAIT"),
                      "torch": torch.__version__, "threads_added": new,
                      "watchdog": any("watchd" in n for n in after),
                      "all_threads": after}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "child":
        child()
    else:
        import subprocess
        rc = 0
        for mode in ("1", "0"):
            env = dict(os.environ, TORCH_NCCL_BLOCKING_WAIT=mode)
            rc |= subprocess.run([sys.executable, __file__, "child"], env=env, timeout=120).returncode
        sys.exit(rc)
