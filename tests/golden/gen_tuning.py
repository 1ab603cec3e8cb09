"""Generate tests/golden/tuning_results.json from the reference's
ControllerTuner (controllers/tuning.py:581-1129): a small random search, its
results file, and a resumed run (`resume_from` that file, more iterations).

Test infrastructure only (build container, reference mounted read-only; the
same no-op `python-dotenv` stand-in as gen_golden.py).  Records both
TuningResult dictionaries (timestamps dropped) and the best-config file.

Usage:  python tests/golden/gen_tuning.py [--out tests/golden]
"""

from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gen_golden import import_reference  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
SPACE = {"q_pos_range": [[5e-5, 5e-5, 10.0], [5e-4, 5e-4, 25.0]],
         "q_vel_range": [[1e-3, 1e-3, 2.0], [1e-2, 1e-2, 8.0]]}
BASE = {"controller_type": "riccati_lqr", "search_space": SPACE, "strategy": "random", "max_iterations": 3,
        "evaluation_episodes": 2, "seed": 5, "target_motion_type": "circular", "episode_length": 2.0}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=HERE)
    args = ap.parse_args()
    import_reference()
    from quadcopter_tracking.controllers.tuning import ControllerTuner, TuningConfig

    out = {"base": BASE}
    with tempfile.TemporaryDirectory() as tmp:
        first = ControllerTuner(TuningConfig.from_dict(dict(BASE, output_dir=os.path.join(tmp, "a")))).tune()
        res_file = glob.glob(os.path.join(tmp, "a", "*_results.json"))[0]
        best_file = glob.glob(os.path.join(tmp, "a", "*_best_config.json"))[0]
        out["first"] = {k: v for k, v in first.to_dict().items() if k != "timestamp"}
        out["first_best_config_file"] = json.load(open(best_file))
        out["first_results_file"] = {k: v for k, v in json.load(open(res_file)).items() if k != "timestamp"}
        resumed = ControllerTuner(TuningConfig.from_dict(dict(BASE, max_iterations=5, resume_from=res_file,
                                                              output_dir=os.path.join(tmp, "b")))).tune()
        out["resumed"] = {k: v for k, v in resumed.to_dict().items() if k not in ("timestamp",)}
        out["resumed"]["config"].pop("resume_from")
        out["resumed"]["config"].pop("output_dir")
        out["first"]["config"].pop("output_dir")
        out["first_results_file"]["config"].pop("output_dir")
    with open(os.path.join(args.out, "tuning_results.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
