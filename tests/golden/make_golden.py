"""Generate the golden one-step fixtures under tests/golden/ (run from the repo root:
``python tests/golden/make_golden.py``).

The reference cannot be run here, so the expected outputs come from the CPU
oracle (oracle/vmas_oracle.py); the fixtures freeze the oracle's answers on non-trivial states so
that later changes to the oracle or the engine are caught ("parity partially pinned": these are
oracle vectors, not reference vectors).

Per scenario: build the env on CPU at 16 envs, take 3 engine steps with seeded random actions
to reach a non-trivial state, then store (inputs = state + agent forces, expected = oracle step,
LIDAR angles + oracle ray distances for every agent sensor).  Plain npz, no pickles.
"""
import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
from oracle import vmas_oracle as O  # noqa: E402
from tests._parity import SCENARIOS, make  # noqa: E402

N_ENVS = 16


def main():
    out_dir = Path(__file__).resolve().parent
    for name, kw, substeps in SCENARIOS:
        env = make(name, kw, substeps, "cpu", num_envs=N_ENVS, seed=7)
        env.seed(7)
        for _ in range(3):
            env.step(env.get_random_actions())
        w = env.world
        snap = O.snapshot(w)
        expected, _ = O.oracle_step(w, snap)
        arrays = {}
        for i, d in snap.items():
            for k, v in d.items():
                arrays[f"in/{i}/{k}"] = v.numpy()
        for i, d in expected.items():
            for k, v in d.items():
                arrays[f"out/{i}/{k}"] = v.numpy()
        ow = O.OracleWorld(w, snap)
        n_lidar = 0
        for agent in w.agents:
            ai = w.entities.index(agent)
            for j, sensor in enumerate(agent.sensors):
                angles = sensor._angles.detach().cpu() + snap[ai]["rot"]
                arrays[f"lidar/{ai}/{j}/angles"] = angles.numpy()
                arrays[f"lidar/{ai}/{j}/dist"] = ow.cast_rays(ai, angles, sensor._max_range, sensor.entity_filter).numpy()
                n_lidar += 1
        meta = {"scenario": name, "kwargs": kw, "substeps": substeps, "num_envs": N_ENVS, "seed": 7,
                "n_entities": len(w.entities), "n_lidar": n_lidar, "torch": torch.__version__}
        arrays["meta"] = np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8)
        np.savez_compressed(out_dir / f"{name}.npz", **arrays)
        print(f"{name}: {len(w.entities)} entities, {n_lidar} lidars")


if __name__ == "__main__":
    main()
