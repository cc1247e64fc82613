"""Do independent branches of a captured HIP graph run concurrently on replay, and what does a
cross-stream edge cost?  Spin kernels (torch.cuda._sleep: one workgroup spinning for N cycles) so
that concurrency, not bandwidth, decides the time.

    python scripts/graph_branch_probe.py
"""
import time

import torch


def replay_ms(g, reps=20):
    g.replay()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) * 1e3 / reps


def main():
    cyc = 200_000  # ~80 us at ~2.4 GHz
    n = 20
    main_s = torch.cuda.Stream()
    side = torch.cuda.Stream()
    res = {}
    # 1. one stream, 2n spins
    g1 = torch.cuda.CUDAGraph()
    with torch.cuda.stream(main_s):
        with torch.cuda.graph(g1, stream=main_s):
            for _ in range(2 * n):
                torch.cuda._sleep(cyc)
    res["serial_2n"] = replay_ms(g1)
    # 2. two branches of n spins each, one fork and one join
    g2 = torch.cuda.CUDAGraph()
    with torch.cuda.stream(main_s):
        with torch.cuda.graph(g2, stream=main_s):
            side.wait_stream(main_s)
            with torch.cuda.stream(side):
                for _ in range(n):
                    torch.cuda._sleep(cyc)
            for _ in range(n):
                torch.cuda._sleep(cyc)
            main_s.wait_stream(side)
    res["branches_n_n"] = replay_ms(g2)
    # 3. 2n spins on one stream with 2n tiny fork/join pairs around them (edge cost)
    g3 = torch.cuda.CUDAGraph()
    with torch.cuda.stream(main_s):
        with torch.cuda.graph(g3, stream=main_s):
            for _ in range(2 * n):
                torch.cuda._sleep(cyc)
                side.wait_stream(main_s)
                with torch.cuda.stream(side):
                    torch.cuda._sleep(10)
                main_s.wait_stream(side)
    res["serial_2n_with_2n_forkjoins"] = replay_ms(g3)
    # 4. short spins: per-node cost on one stream
    g4 = torch.cuda.CUDAGraph()
    with torch.cuda.stream(main_s):
        with torch.cuda.graph(g4, stream=main_s):
            for _ in range(200):
                torch.cuda._sleep(10)
    res["200_tiny_nodes"] = replay_ms(g4)
    g5 = torch.cuda.CUDAGraph()
    with torch.cuda.stream(main_s):
        with torch.cuda.graph(g5, stream=main_s):
            for k in range(100):
                side.wait_stream(main_s)
                with torch.cuda.stream(side):
                    torch.cuda._sleep(10)
                main_s.wait_stream(side)
                torch.cuda._sleep(10)
    res["100_tiny_pingpong_pairs"] = replay_ms(g5)
    for k, v in res.items():
        print(f"{k:32s} {v:8.3f} ms", flush=True)


if __name__ == "__main__":
    main()
