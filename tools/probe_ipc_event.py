#!/usr/bin/env python3
"""Probe: can two processes on this box share a HIP event (hipIpcGetEventHandle /
hipIpcOpenEventHandle via torch.cuda.Event(interprocess=True)) and order a stream
in one process after work recorded in the other?  Used by the async PS's
device-side hand-off (parallel/async_ps.py)."""
import os
import sys
import time

import torch
import torch.multiprocessing as mp


def child(q_h, q_back):
    d = torch.device("cuda", 0)
    torch.cuda.set_device(d)
    h, buf_h = q_h.get()
    ev = torch.cuda.Event.from_ipc_handle(d, h)
    buf = buf_h
    s = torch.cuda.current_stream()
    s.wait_event(ev)          # device-side wait on the parent's recorded work
    v = float(buf[-1].item())  # must see the value the parent's kernel wrote before recording
    q_back.put(v)


def main():
    mp.set_start_method("spawn")
    d = torch.device("cuda", 0)
    torch.cuda.set_device(d)
    ev = torch.cuda.Event(interprocess=True)
    buf = torch.zeros(1 << 24, device=d)
    q_h, q_back = mp.Queue(), mp.Queue()
    p = mp.Process(target=child, args=(q_h, q_back))
    p.start()
    # a long kernel chain, then the marker value, then the record: the child must see 7
    for _ in range(20):
        buf.mul_(1.0001)
    buf[-1] = 7.0
    ev.record()
    q_h.put((ev.ipc_handle(), buf))
    v = q_back.get(timeout=120)
    p.join(timeout=60)
    print(f"ipc event probe: child saw {v} (want 7.0) exit {p.exitcode}", flush=True)
    return 0 if v == 7.0 and p.exitcode == 0 else 1


if __name__ == "__main__":
    sys.exit(main())
