"""Do the parallel branches of a captured hipGraph run concurrently?  (round 5 found that the
fp32 conv2 weight gradient forked onto a side stream gained nothing in the replayed step,
profiles/r5ab_fp32_side_stream_reverted.txt.)  Two ~40 us spin kernels (torch.cuda._sleep) on
two streams -- eager, and captured as fork / join branches of one graph -- timed against the
same two kernels on one stream.  Run it under different HIP graph settings, e.g.
    python scripts/exp/graph_branches.py
    DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 python scripts/exp/graph_branches.py
prints us per replay: serial ~2x the single kernel, overlapped ~1x."""
import os
import time

import torch

CYC = int(os.environ.get("SPIN_CYCLES", "100000"))  # ~40 us at ~2.4 GHz


def two_streams(s1, s2):
    cur = torch.cuda.current_stream()
    s1.wait_stream(cur)
    s2.wait_stream(cur)
    with torch.cuda.stream(s1):
        torch.cuda._sleep(CYC)
    with torch.cuda.stream(s2):
        torch.cuda._sleep(CYC)
    cur.wait_stream(s1)
    cur.wait_stream(s2)


def one_stream():
    torch.cuda._sleep(CYC)
    torch.cuda._sleep(CYC)


def timed(fn, n=50):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e6


def main():
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    single = timed(lambda: torch.cuda._sleep(CYC))
    rows = [("one kernel", single), ("eager, one stream", timed(one_stream)),
            ("eager, two streams", timed(lambda: two_streams(s1, s2)))]
    for name, body in (("graph, one stream", one_stream), ("graph, fork/join branches", lambda: two_streams(s1, s2))):
        g = torch.cuda.CUDAGraph()
        cs = torch.cuda.Stream()
        cs.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(cs):
            body()
        torch.cuda.current_stream().wait_stream(cs)
        torch.cuda.synchronize()
        with torch.cuda.graph(g):
            body()
        rows.append((name, timed(g.replay)))
    env = {k: os.environ[k] for k in os.environ if k.startswith(("DEBUG_HIP", "DEBUG_CLR", "GPU_MAX_HW"))}
    print(f"env {env}", flush=True)
    for name, us in rows:
        print(f"  {name:28s} {us:8.1f} us  ({us / single:4.2f} x one kernel)", flush=True)


if __name__ == "__main__":
    main()
