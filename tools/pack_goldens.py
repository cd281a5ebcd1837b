"""Packs the reference outputs the survey produced in this container
(/tmp/scenes, see tests/golden/README.md) into tests/golden/. Run once, here;
the GPU box and later rounds only read the packed files."""
import json
import os
import sys

import numpy as np

SRC = sys.argv[1] if len(sys.argv) > 1 else "/tmp/scenes"
DST = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden")


def read_tga(path):
    d = np.fromfile(path, np.uint8)
    idl, w, h = int(d[0]), int(d[12]) | int(d[13]) << 8, int(d[14]) | int(d[15]) << 8
    assert d[2] == 2 and d[16] == 24, "uncompressed 24-bit TGA expected"
    px = d[18 + idl:18 + idl + w * h * 3].reshape(h, w, 3)[:, :, ::-1]  # BGR -> RGB
    if not (d[17] & 0x20):  # bottom-left origin
        px = px[::-1]
    return np.ascontiguousarray(px)


frames = {
    "cornell_dl_512_4spp_t1": "o_cornell_dl.tga",
    "cornell_pt_256_16spp_t1": "o_cornell_pt.tga",
    "bumpy1m_480x270_4spp_t1": "o_bumpy1m_t1.tga",
    "cornell_pt_1024_64spp_t8": "o_cfg2.tga",
}
for k, f in frames.items():
    np.savez_compressed(os.path.join(DST, k + ".npz"), rgb8=read_tga(os.path.join(SRC, f)))
crop = np.fromfile(os.path.join(SRC, "crop.f32"), np.float32).reshape(48, 64, 4)
np.save(os.path.join(DST, "cornell_pt_256_16spp_crop_x100_y120_64x48.npy"), crop)
print("packed", sorted(os.listdir(DST)))
