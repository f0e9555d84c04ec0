#!/usr/bin/env python3
"""Probe 3: an interprocess event re-recorded MANY times by its producer while an
independent consumer process waits on it at its own pace (the async PS's
"update recorded" event under two pushing workers)."""
import base64
import datetime
import socket
import subprocess
import sys

import torch
import torch.distributed as dist

N = 300


def consumer(port):
    torch.cuda.set_device(0)
    st = dist.TCPStore("127.0.0.1", port, 2, False, timeout=datetime.timedelta(seconds=60))
    ev = torch.cuda.Event.from_ipc_handle(torch.device("cuda", 0), base64.b64decode(st.get("ev")))
    y = torch.zeros(1 << 22, device="cuda")
    bad = 0
    for i in range(N):
        try:
            torch.cuda.current_stream().wait_event(ev)
        except Exception as e:  # noqa: BLE001
            bad += 1
            if bad < 4:
                print(f"consumer: wait {i} failed: {e}".splitlines()[0], flush=True)
        y.add_(1)
        if i % 7 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    print(f"consumer: {N} waits, {bad} failed", flush=True)
    st.set("done", "1")
    return 1 if bad else 0


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "consumer":
        return consumer(int(sys.argv[2]))
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    torch.cuda.set_device(0)
    st = dist.TCPStore("127.0.0.1", port, 2, True, timeout=datetime.timedelta(seconds=60), wait_for_workers=False)
    p = subprocess.Popen([sys.executable, __file__, "consumer", str(port)])
    ev = torch.cuda.Event(interprocess=True)
    x = torch.zeros(1 << 22, device="cuda")
    x.add_(1)
    ev.record()
    st.set("ev", base64.b64encode(bytes(ev.ipc_handle())).decode())
    for i in range(4 * N):
        x.add_(1)
        ev.record()
    st.get("done")
    rc = p.wait(timeout=60)
    print("producer: consumer exit", rc, flush=True)
    return rc


if __name__ == "__main__":
    sys.exit(main())
