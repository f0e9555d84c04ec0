#!/usr/bin/env python3
"""Probe 2: the IPC event shared between two INDEPENDENT processes (Popen, not a
torch.multiprocessing child) through a TCPStore, as the async PS replicas do;
then the producer re-records it after more work and the consumer waits again."""
import base64
import datetime
import os
import subprocess
import sys

import torch
import torch.distributed as dist


def consumer(port):
    torch.cuda.set_device(0)
    st = dist.TCPStore("127.0.0.1", port, 2, False, timeout=datetime.timedelta(seconds=60))
    ev = torch.cuda.Event.from_ipc_handle(torch.device("cuda", 0), base64.b64decode(st.get("ev")))
    print("consumer: opened", flush=True)
    torch.cuda.current_stream().wait_event(ev)
    torch.cuda.synchronize()
    st.set("c1", "1")
    st.get("p2")
    torch.cuda.current_stream().wait_event(ev)
    torch.cuda.synchronize()
    print("consumer: waited twice ok", flush=True)
    st.set("c2", "1")


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "consumer":
        consumer(int(sys.argv[2]))
        return 0
    import socket
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    torch.cuda.set_device(0)
    st = dist.TCPStore("127.0.0.1", port, 2, True, timeout=datetime.timedelta(seconds=60), wait_for_workers=False)
    p = subprocess.Popen([sys.executable, __file__, "consumer", str(port)])
    ev = torch.cuda.Event(interprocess=True)
    x = torch.zeros(1 << 20, device="cuda")
    x.add_(1)
    ev.record()
    st.set("ev", base64.b64encode(bytes(ev.ipc_handle())).decode())
    st.get("c1")
    x.add_(1)
    ev.record()
    st.set("p2", "1")
    st.get("c2")
    rc = p.wait(timeout=60)
    print("producer: consumer exit", rc, flush=True)
    return rc


if __name__ == "__main__":
    sys.exit(main())
