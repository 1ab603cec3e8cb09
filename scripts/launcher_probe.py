#!/usr/bin/env python3
"""What bench.py's launcher sees on this machine, without touching HIP: the
KFD GPU nodes, their render nodes and whether this process may open them,
the *_VISIBLE_DEVICES lists, and bench.visible_gpu_count()."""

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

base = "/sys/class/kfd/kfd/topology/nodes"
nodes = []
for node in sorted(os.listdir(base)) if os.path.isdir(base) else []:
    try:
        props = dict(line.split(" ", 1) for line in open(os.path.join(base, node, "properties")).read().splitlines()
                     if " " in line)
    except OSError:
        continue
    if int(props.get("simd_count", "0")) > 0:
        render = f"/dev/dri/renderD{int(props.get('drm_render_minor', '-1'))}"
        nodes.append({"node": node, "render": render, "exists": os.path.exists(render),
                      "rw": os.access(render, os.R_OK | os.W_OK)})
print(json.dumps({"gpu_nodes": nodes, "visible_gpu_count": bench.visible_gpu_count(),
                  "env": {k: os.environ.get(k) for k in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES",
                                                         "CUDA_VISIBLE_DEVICES")},
                  "torch_loaded": "torch" in sys.modules}))
