"""Which HIP event queries fail while a stream is capturing (the RCCL watchdog abort).

No process group is involved: the probe reproduces, on its own, the query the ProcessGroupNCCL watchdog makes
(``WorkNCCL::finishedGPUExecutionInternal`` -> ``at::cuda::CUDAEvent::query`` -> ``hipEventQuery``) from another
thread while the main thread captures a graph in ``thread_local`` mode.  Three events, all recorded EAGERLY and
complete (device synchronised) before the capture starts:

* ``eager_on_capturing_stream``: recorded on the stream that is then captured (where an async_op=False collective of
  a warm-up step records its Work's end event);
* ``eager_on_other_stream``: recorded on a stream that never captures;
* ``eager_on_capturing_stream_after_end``: the first event again, queried after the capture has ended.

Output: one JSON line (``--out`` also writes it to a file).  Usage: ``python tools/captured_event_probe.py``.
"""
import argparse
import json
import threading

import torch


def _query(e):
    try:
        return "complete" if e.query() else "not_ready"
    except Exception as ex:   # torch raises on any status other than success / not-ready
        return "raised: " + str(ex).splitlines()[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    s, t = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    x = torch.ones(1 << 16, device=dev)
    e_s, e_t = torch.cuda.Event(), torch.cuda.Event()
    with torch.cuda.stream(s):
        x.mul_(2)
        e_s.record(s)
    with torch.cuda.stream(t):
        x.add_(0)
        e_t.record(t)
    torch.cuda.synchronize()
    res = {"before_capture": {"eager_on_capturing_stream": _query(e_s), "eager_on_other_stream": _query(e_t)}}
    during = {}

    def poll():   # the watchdog's view: another host thread, no capture of its own
        during["eager_on_capturing_stream"] = _query(e_s)
        during["eager_on_other_stream"] = _query(e_t)

    g = torch.cuda.CUDAGraph()
    try:
        with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
            y = x * 3
            th = threading.Thread(target=poll)
            th.start()
            th.join()
            y.add_(1)
        res["capture_end"] = "ok"
    except Exception as ex:
        res["capture_end"] = "raised: " + str(ex).splitlines()[0]
    res["during_capture_from_other_thread"] = during
    torch.cuda.synchronize()
    res["eager_on_capturing_stream_after_end"] = _query(e_s)
    res["torch"] = torch.__version__
    res["hip"] = torch.version.hip
    line = json.dumps(res)
    print(line, flush=True)
    if a.out:
        with open(a.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
