"""Generate tests/golden/trainer_epochs.json from the reference's
`Trainer._evaluate_epoch` (train.py:578-652), the classical controllers'
evaluation epoch — the third caller of the hot path.

Test infrastructure only (build container, reference mounted read-only; the
same no-op `python-dotenv` stand-in as gen_golden.py).  For every scenario it
builds the reference Trainer from a TrainingConfig, runs `_evaluate_epoch` at
the listed epochs and records the returned dict, and — with the reference's
own env and a fresh reference controller, seeds env_seed + epoch * 1000 + ep
— each episode's reward sum, last-step info["on_target_ratio"] and
info["tracking_error"] and step count.  The generator asserts that np.mean of
those per-episode values is the Trainer's own return, bit for bit.

Usage:  python tests/golden/gen_trainer.py [--out tests/golden]
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gen_golden import import_reference  # noqa: E402

SCENARIOS = [
    {"name": "riccati_circular_full", "controller": "riccati_lqr", "ctl": {},
     "motion": "circular", "env_seed": 42, "episode_length": 30.0, "target_radius": 0.5,
     "episodes_per_epoch": 3, "max_steps_per_episode": 3000, "epochs": [0, 2]},
    {"name": "pid_linear_truncated", "controller": "pid", "ctl": {"kp_pos": [0.02, 0.02, 4.5]},
     "motion": "linear", "env_seed": 7, "episode_length": 30.0, "target_radius": 0.5,
     "episodes_per_epoch": 3, "max_steps_per_episode": 500, "epochs": [1]},
    {"name": "lqr_sinusoidal_short", "controller": "lqr", "ctl": {},
     "motion": "sinusoidal", "env_seed": 11, "episode_length": 5.0, "target_radius": 0.3,
     "episodes_per_epoch": 3, "max_steps_per_episode": 3000, "epochs": [2]},
    {"name": "riccati_lqi_ff_figure8", "controller": "riccati_lqr",
     "ctl": {"use_lqi": True, "q_int": [1e-3, 1e-3, 1e-2], "feedforward_enabled": True,
             "ff_velocity_gain": 0.1, "ff_acceleration_gain": 0.05},
     "motion": "figure8", "env_seed": 3, "episode_length": 30.0, "target_radius": 0.5,
     "episodes_per_epoch": 2, "max_steps_per_episode": 1200, "epochs": [0]},
    {"name": "riccati_stationary_ten", "controller": "riccati_lqr", "ctl": {"q_pos": [1e-4, 1e-4, 20.0]},
     "motion": "stationary", "env_seed": 100, "episode_length": 30.0, "target_radius": 0.5,
     "episodes_per_epoch": 10, "max_steps_per_episode": 300, "epochs": [5]},
]


def make_controller(qt, kind, cfg):
    from quadcopter_tracking.controllers import LQRController, PIDController
    from quadcopter_tracking.controllers.riccati_lqr import RiccatiLQRController

    return {"pid": PIDController, "lqr": LQRController, "riccati_lqr": RiccatiLQRController}[kind](config=dict(cfg))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.dirname(os.path.abspath(__file__)))
    args = ap.parse_args()
    qt = import_reference()
    from quadcopter_tracking.env import QuadcopterEnv
    from quadcopter_tracking.env.config import EnvConfig
    from quadcopter_tracking.train import Trainer, TrainingConfig

    out = []
    for s in SCENARIOS:
        with tempfile.TemporaryDirectory() as tmp:
            tc = TrainingConfig(controller=s["controller"], episodes_per_epoch=s["episodes_per_epoch"],
                                max_steps_per_episode=s["max_steps_per_episode"], env_seed=s["env_seed"],
                                target_motion_type=s["motion"], episode_length=s["episode_length"],
                                target_radius=s["target_radius"], checkpoint_dir=os.path.join(tmp, "ck"),
                                log_dir=os.path.join(tmp, "logs"), device="cpu")
            tc.full_config = {s["controller"]: dict(s["ctl"])}
            trainer = Trainer(tc)
            epochs = []
            for epoch in s["epochs"]:
                trainer.current_epoch = epoch
                res = trainer._evaluate_epoch()
                # the same episodes with the reference's env and a fresh controller per episode
                env_cfg = EnvConfig()
                env_cfg.seed = s["env_seed"]
                env_cfg.simulation.max_episode_time = s["episode_length"]
                env_cfg.target.motion_type = s["motion"]
                env_cfg.success_criteria.target_radius = s["target_radius"]
                env = QuadcopterEnv(config=env_cfg)
                rew, ratio, err, steps = [], [], [], []
                for ep in range(s["episodes_per_epoch"]):
                    obs = env.reset(seed=s["env_seed"] + epoch * 1000 + ep)
                    ctl = make_controller(qt, s["controller"], s["ctl"])
                    done, step, rs, info = False, 0, [], {}
                    while not done and step < s["max_steps_per_episode"]:
                        obs, r, done, info = env.step(ctl.compute_action(obs))
                        rs.append(r)
                        step += 1
                    rew.append(sum(rs))
                    ratio.append(info.get("on_target_ratio", 0.0))
                    err.append(info.get("tracking_error", 0.0))
                    steps.append(step)
                assert float(np.mean(rew)) == float(res["mean_reward"]), (s["name"], epoch)
                assert float(np.mean(ratio)) == float(res["mean_on_target_ratio"]), (s["name"], epoch)
                assert float(np.mean(err)) == float(res["mean_tracking_error"]), (s["name"], epoch)
                epochs.append({"epoch": epoch, "result": {k: float(v) for k, v in res.items()},
                               "episode_reward": [float(v) for v in rew],
                               "episode_on_target_ratio": [float(v) for v in ratio],
                               "episode_tracking_error": [float(v) for v in err], "episode_steps": steps})
            out.append({**s, "results": epochs})
            print(s["name"], [e["result"] for e in epochs], flush=True)
    path = os.path.join(args.out, "trainer_epochs.json")
    with open(path, "w") as fh:
        json.dump({"source": "reference Trainer._evaluate_epoch (train.py:578-652)", "scenarios": out}, fh,
                  indent=1)
    print("wrote", path)


if __name__ == "__main__":
    main()
