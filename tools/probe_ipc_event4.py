#!/usr/bin/env python3
"""Probe 4: interprocess events in strict alternation (record, then the other process
waits, then the next record) for many rounds, in both directions at once — the async
PS's per-(worker, PS) "mailbox written" / "update done" events."""
import base64
import datetime
import socket
import subprocess
import sys

import torch
import torch.distributed as dist

N = 500


def side(port, me):
    torch.cuda.set_device(0)
    st = dist.TCPStore("127.0.0.1", port, 2, me == 0, timeout=datetime.timedelta(seconds=120),
                       wait_for_workers=False)
    mine = torch.cuda.Event(interprocess=True)
    x = torch.zeros(1 << 22, device="cuda")
    x.add_(1)
    mine.record()
    st.set(f"ev{me}", base64.b64encode(bytes(mine.ipc_handle())).decode())
    other = torch.cuda.Event.from_ipc_handle(torch.device("cuda", 0), base64.b64decode(st.get(f"ev{1 - me}")))
    bad = 0
    for i in range(N):
        if me == 0:  # record, tell; wait for the other's record
            x.add_(1)
            mine.record()
            st.set(f"a{i}", "1")
            st.get(f"b{i}")
            try:
                torch.cuda.current_stream().wait_event(other)
            except Exception as e:  # noqa: BLE001
                bad += 1
                if bad < 3:
                    print(f"side 0: wait {i}: {str(e).splitlines()[0]}", flush=True)
        else:
            st.get(f"a{i}")
            try:
                torch.cuda.current_stream().wait_event(other)
            except Exception as e:  # noqa: BLE001
                bad += 1
                if bad < 3:
                    print(f"side 1: wait {i}: {str(e).splitlines()[0]}", flush=True)
            x.add_(1)
            mine.record()
            st.set(f"b{i}", "1")
    torch.cuda.synchronize()
    print(f"side {me}: {N} rounds, {bad} failed waits", flush=True)
    st.set(f"end{me}", "1")
    st.get(f"end{1 - me}")
    return 1 if bad else 0


def main():
    if len(sys.argv) > 2:
        return side(int(sys.argv[2]), int(sys.argv[1]))
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    p = subprocess.Popen([sys.executable, __file__, "1", str(port)])
    rc0 = side(port, 0)
    rc1 = p.wait(timeout=120)
    return rc0 or rc1


if __name__ == "__main__":
    sys.exit(main())
