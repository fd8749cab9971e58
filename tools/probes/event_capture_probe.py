"""When does hipEventQuery answer hipErrorCapturedEvent ("operation not permitted on an event last
recorded in a capturing stream")?  The RCCL watchdog polls the end event of every eager collective with
it and aborts the process on that error (VERDICT r5 "What's weak" 2).  Each case runs in its own
subprocess (a refused query can invalidate a capture); the query always comes from a second thread, as
the watchdog's does.

  a  E recorded eagerly on S (complete); S captures; query E during the capture
  b  E recorded eagerly on S; stream C waits on E; C captures; query E during the capture
  c  E recorded on S inside a capture of S; query E after the capture ended
  d  as c, then E recorded again eagerly on S; query E
  e  as c, then E destroyed; a new event recorded eagerly on another stream T; query it
  f  E recorded eagerly on S; an unrelated stream U captures; query E during the capture

usage: python tools/probes/event_capture_probe.py            (runs every case, prints one line each)"""
import subprocess
import sys
import threading

import torch


def _query_in_thread(e):
    out = {}

    def poll():
        try:
            out["r"] = e.query()
        except Exception as ex:  # noqa: BLE001
            out["r"] = "ERROR " + str(ex).splitlines()[0]

    t = threading.Thread(target=poll)
    t.start()
    t.join()
    return out["r"]


def case(name):
    dev = torch.device("cuda", 0)
    S, C, T, U = (torch.cuda.Stream(dev) for _ in range(4))
    x = torch.zeros(1024, device=dev)
    e = torch.cuda.Event()
    g = torch.cuda.CUDAGraph()
    res = None
    if name in ("a", "b", "f"):
        with torch.cuda.stream(S):
            x.add_(1)
            e.record(S)
        torch.cuda.synchronize()
        cap = {"a": S, "b": C, "f": U}[name]
        if name == "b":
            C.wait_event(e)
        with torch.cuda.graph(g, stream=cap, capture_error_mode="thread_local"):
            x.add_(1)
            res = _query_in_thread(e)
            x.add_(1)
    else:
        with torch.cuda.graph(g, stream=S, capture_error_mode="thread_local"):
            x.add_(1)
            e.record(S)
        torch.cuda.synchronize()
        if name == "c":
            res = _query_in_thread(e)
        elif name == "d":
            with torch.cuda.stream(S):
                x.add_(1)
                e.record(S)
            torch.cuda.synchronize()
            res = _query_in_thread(e)
        else:
            del e
            e2 = torch.cuda.Event()
            with torch.cuda.stream(T):
                x.add_(1)
                e2.record(T)
            torch.cuda.synchronize()
            res = _query_in_thread(e2)
    print(f"case {name}: query -> {res}", flush=True)


def main():
    if len(sys.argv) > 1:
        case(sys.argv[1])
        return
    for name in "abcdef":
        p = subprocess.run([sys.executable, __file__, name], capture_output=True, text=True, timeout=120)
        lines = [ln for ln in (p.stdout + p.stderr).splitlines() if ln.startswith("case") or "Error" in ln]
        print(f"[{name}] rc={p.returncode} " + " | ".join(lines[:3]), flush=True)


if __name__ == "__main__":
    main()
