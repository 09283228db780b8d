"""Builds tests/golden/lm_test_bboxes_yolov3.npz from the reference's detection fixture
dataset/linemod/dataset_config/test_bboxes/bbox_yolov3_all.json (data, not code: one
[x, y, w, h] YOLOv3 box per LineMOD test frame). Run here (the reference is not on the GPU box):

    python tests/golden/make_bbox_fixture.py /root/reference
"""
import json
import os
import sys

import numpy as np

ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
src = os.path.join(ref, "dataset/linemod/dataset_config/test_bboxes/bbox_yolov3_all.json")
d = json.load(open(src))
keys = sorted(d, key=lambda k: (int(k.split("/")[0]), int(k.split("/")[1])))
rows = []
for k in keys:
    for det in d[k]:
        rows.append([det["obj_id"], *det["bbox_est"]])
a = np.asarray(rows, dtype=np.float64)
box = a[:, 1:].astype(np.float32)
assert np.array_equal(box.astype(np.float64), a[:, 1:]), "boxes are float32 values"
out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lm_test_bboxes_yolov3.npz")
np.savez_compressed(out, obj_id=a[:, 0].astype(np.int16), bbox=box)
print(out, a.shape)
