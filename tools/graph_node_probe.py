"""Cost of one small dependent kernel inside a replayed HIP graph (the scenario tensor program
of graph mode: ~40-300 elementwise kernels on [32768] fp32 tensors per step).

Prints one JSON line: microseconds per node for a chain of N dependent elementwise kernels,
replayed as one graph, plus the same chain launched eagerly.  Run it under different runtime
environment settings (tools/graph_node_ab.sh) to see what the dependent-launch cost depends on.
"""
import json
import os
import sys
import time

import torch


def main():
    n_nodes = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 32768
    dev = torch.device("cuda:0")
    x = torch.rand(B, device=dev)
    y = torch.rand(B, device=dev)

    def chain():
        a = x
        for i in range(n_nodes):
            a = a * 0.999 + y if i % 2 else a - y
        return a

    for _ in range(3):
        chain()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        chain()
    torch.cuda.synchronize()
    eager_us = (time.perf_counter() - t0) / 10 / (n_nodes * 1.5) * 1e6  # a*c + y is 2 kernels

    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        chain()
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(g):
        chain()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    reps = 50
    t0 = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    graph_us = (time.perf_counter() - t0) / reps / (n_nodes * 1.5) * 1e6
    env = {k: v for k, v in os.environ.items() if k.startswith(("HIP_", "DEBUG_CLR", "GPU_", "AMD_", "ROC_", "HSA_"))}
    print(json.dumps({"nodes": int(n_nodes * 1.5), "B": B, "graph_us_per_node": round(graph_us, 3),
                      "eager_us_per_kernel": round(eager_us, 3), "env": env}), flush=True)


if __name__ == "__main__":
    main()
