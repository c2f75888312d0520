"""Diagnostic (GPU): where the Euclidean-HOCBF lattice step's solves go at the cfg4 shape.

Steps a 1024 x 1024 lattice swarm in HOCBF mode and prints, at a few timesteps, the histograms of
the neighbour count and of the relaxation count (status >> 8) over the egos, so the main kernel's
per-lane solve length can be read off.  `python tools/diag_hocbf.py [steps]`.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from cbf_amd import scenarios, swarm
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    W = H = 1024
    S = swarm.LatticeSwarm(scenarios.lattice(W, H, seed=0, spacing=0.145), W, H, gain=scenarios.LATTICE_GAIN,
                           barrier="euclidean_hocbf")
    for t in range(steps):
        S.step()
        if t in (5, 15, 25, steps - 1):
            torch.cuda.synchronize()
            st = S.status.cpu()
            cnt = S.nbr_count.cpu()
            code = st & 0xFF
            it = st >> 8
            print(f"timestep {t}: status codes {dict(zip(*[v.tolist() for v in torch.unique(code, return_counts=True)]))}")
            print(f"  neighbours {dict(zip(*[v.tolist() for v in torch.unique(cnt, return_counts=True)]))}")
            print(f"  relaxations {dict(zip(*[v.tolist() for v in torch.unique(it, return_counts=True)]))}")
            m8 = (cnt > 0) & (cnt <= 8)
            print(f"  relaxations (m <= 8) mean {it[m8].double().mean().item():.3f}", flush=True)


if __name__ == "__main__":
    main()
