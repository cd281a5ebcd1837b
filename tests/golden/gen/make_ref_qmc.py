"""Writes tests/golden/ref_qmc.npz: inputs and the reference's own outputs of
its header-only QMC / fast-math layer, compiled HERE from
/root/reference/include by oracle/ref.mk (oracle/_ref/ref_check, survey-build
flags -O3 -ffast-math -DFAST_MATH -DFAST_TRIG).

Functions (reference file:line): RI_vdC / RI_S / RI_LP / fnv_32a_buf
(utilities/mcqmc.h:100,110,117,155), Halton::setStart + getNext bases 2, 3, 5
(mcqmc.h:29-94), fSin / fCos / fExp2 (utilities/mathOptimizations.h:249,273,
100), Round2Int / Floor2Int (utilities/math_utils.h:60,80).

Run in the build container (needs /root/reference):
    make -C oracle -f ref.mk && python tests/golden/gen/make_ref_qmc.py
The GPU box has no reference: tests read the committed .npz.
"""
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.abspath(os.path.join(HERE, "..", "..", ".."))
EXE = os.path.join(ROOT, "oracle", "_ref", "ref_check")

ARRAYS = {  # name: dtype
    "u_in": np.uint32, "u_r": np.uint32, "ri_vdc": np.uint32, "ri_s": np.uint32, "ri_lp": np.uint32,
    "fnv": np.uint32, "f_in": np.float32, "fsin": np.uint32, "fcos": np.uint32, "hal_start": np.uint32,
    "hal2": np.float32, "hal3": np.float32, "hal5": np.float32, "e_in": np.float32, "fexp2": np.uint32,
    "d_in": np.float64, "round2int": np.int32, "floor2int": np.int32,
}


def main():
    if not os.path.exists(EXE):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "-f", "ref.mk"], check=True)
    with tempfile.TemporaryDirectory() as d:
        subprocess.run([EXE, "fixtures", d], check=True)
        out = {k: np.fromfile(os.path.join(d, k + ".bin"), dtype=t) for k, t in ARRAYS.items()}
    for b in (2, 3, 5):
        out["hal%d" % b] = out["hal%d" % b].reshape(-1, 8)
    dst = os.path.join(ROOT, "tests", "golden", "ref_qmc.npz")
    np.savez_compressed(dst, **out)
    print(dst, {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    sys.exit(main())
