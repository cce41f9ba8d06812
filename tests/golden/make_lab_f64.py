"""The LearnableAffineBlock scalar gradients of the N full-step fixture (train_full_n_b2.npz) in
float64: the oracle (oracle/train_cpu.py via tests/test_train_oracle.py::oracle_train_step_full,
pinned to the reference's fp32 step) run in double precision on the fixture's inputs and DN
draws. A LAB scalar's gradient is a sum over a whole feature map that largely cancels, so fp32
(the reference's own step included) carries rounding noise of up to ~14 % there; the GPU test
judges the HIP step's LAB gradients against these values instead of the fp32 fixture.

    python tests/golden/make_lab_f64.py    # -> tests/golden/train_full_n_b2_lab_f64.npz
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, os.path.dirname(HERE))


def main():
    from test_train_oracle import oracle_train_step_full
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    g = np.load(os.path.join(HERE, "train_full_n_b2.npz"))
    names = sorted(f[:-len("__val")] for f in g.files
                   if f.startswith("grad.") and f.endswith("__val") and f.endswith(("lab.scale__val", "lab.bias__val")))
    _, grads, _, _, _ = oracle_train_step_full("n", g, dtype=torch.float64)
    vals = np.array([float(grads[n].reshape(-1)[0]) for n in names], dtype=np.float64)
    np.savez(os.path.join(HERE, "train_full_n_b2_lab_f64.npz"), names=np.array(names), f64=vals,
             ref_fp32=np.array([float(g[n + "__val"][0]) for n in names], dtype=np.float64))
    print(len(names), "LAB scalars")


if __name__ == "__main__":
    main()
