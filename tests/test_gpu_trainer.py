"""The trainer's classical evaluation epoch (quadtrack.train.evaluate_epoch,
one qt_rollout_rewards launch per epoch) against the reference's own
Trainer._evaluate_epoch (train.py:578-652), run by
tests/golden/gen_trainer.py into trainer_epochs.json: per-episode reward sums,
last-step info on-target ratios and tracking errors, step counts (exact), and
the epoch means.

Tolerance: 1e-8 relative (and 1e-8 absolute) on every value — the
trajectories differ from the reference's only by the DARE gains' sub-ulp
difference (scipy QZ vs the doubling algorithm) — and step counts and
on-target ratios (integer counts) exactly."""

import json
import os
from types import SimpleNamespace

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

FIX = json.load(open(os.path.join(GOLDEN, "trainer_epochs.json")))["scenarios"]
CASES = [(s, e) for s in FIX for e in s["results"]]


@pytest.mark.parametrize("s,ep", CASES, ids=[f"{s['name']}-epoch{e['epoch']}" for s, e in CASES])
def test_evaluate_epoch_matches_reference_trainer(s, ep):
    from quadtrack import _abi
    from quadtrack.train import evaluate_epoch

    _abi.require_gpu()
    cfg = SimpleNamespace(controller=s["controller"], episodes_per_epoch=s["episodes_per_epoch"],
                          max_steps_per_episode=s["max_steps_per_episode"], env_seed=s["env_seed"],
                          target_motion_type=s["motion"], episode_length=s["episode_length"],
                          target_radius=s["target_radius"], full_config={s["controller"]: s["ctl"]})
    r = evaluate_epoch(cfg, epoch=ep["epoch"])
    np.testing.assert_array_equal(r.episode_steps.cpu().numpy(), ep["episode_steps"])
    np.testing.assert_array_equal(r.episode_on_target_ratio.cpu().numpy(), ep["episode_on_target_ratio"])
    np.testing.assert_allclose(r.episode_reward.cpu().numpy(), ep["episode_reward"], rtol=1e-8, atol=1e-8)
    np.testing.assert_allclose(r.episode_tracking_error.cpu().numpy(), ep["episode_tracking_error"], rtol=1e-8,
                               atol=1e-8)
    got = r.as_dict()
    assert got["difficulty"] == 1.0
    assert got["mean_on_target_ratio"] == ep["result"]["mean_on_target_ratio"]
    for k in ("mean_reward", "mean_tracking_error"):
        np.testing.assert_allclose(got[k], ep["result"][k], rtol=1e-8, atol=1e-8, err_msg=k)


def test_evaluate_epoch_means_are_numpy_means():
    """The epoch means are np.mean of the per-episode values, bit for bit
    (qt_summary_numpy), at 10 episodes (numpy's 8-accumulator leaf) and 37."""
    from quadtrack import _abi
    from quadtrack.train import evaluate_epoch

    _abi.require_gpu()
    for n in (10, 37):
        r = evaluate_epoch(controller="riccati_lqr", episodes_per_epoch=n, max_steps_per_episode=200,
                           target_motion_type="sinusoidal", env_seed=5)
        assert r.mean_reward == float(np.mean(r.episode_reward.cpu().numpy()))
        assert r.mean_on_target_ratio == float(np.mean(r.episode_on_target_ratio.cpu().numpy()))
        assert r.mean_tracking_error == float(np.mean(r.episode_tracking_error.cpu().numpy()))


@pytest.mark.parametrize("controller,motion", [("riccati_lqr", "circular"), ("lqi", "sinusoidal"),
                                               ("pid", "linear"), ("lqr", "figure8")])
def test_rewards_fast_flavour_matches_exact(controller, motion):
    """qt_rollout_rewards on the yaw-at-rest fast flavour (rewards telescoped
    from its pre-step tracking-error sums) against the exact step, which
    accumulates -(post-step error) per step.  The exact run starts every
    episode with a 1e-300 rad/s yaw rate: no lane then passes the yaw-at-rest
    wave test, every wave goes to the exact pass, and the trajectories differ
    by ~1e-300.  Reward sums and last errors within 1e-9, step counts and
    on-target counts exact — in one launch and in three uneven chunks."""
    import torch

    from quadtrack import _abi, core
    from quadtrack.controllers import batched_controller
    from quadtrack.rollout import build_batch
    from quadtrack.train import env_config_for

    dev = _abi.require_gpu()
    cfg = env_config_for(7, motion, 12.0)
    env = cfg.to_params()
    n = 300
    ctl = batched_controller(controller, {}, device=dev)
    batch = build_batch(ctl, cfg, n, seeds=np.arange(n))
    out = []
    for exact, chunks in ((False, [1200]), (False, [401, 555, 244]), (True, [1200])):
        st = core.RolloutState.empty(n, dev)
        core.reset(env, batch, st)
        if exact:
            st.x[11] = 1e-300
        reward = torch.zeros(2, n, dtype=torch.float64, device=dev)
        for k in chunks:
            core.rollout_rewards(env, ctl.ctrl, core.criteria(), batch, st, k, reward)
        out.append((reward.cpu().numpy(), st.acc.cpu().numpy()))
    (r0, a0), (r1, a1), (re, ae) = out
    assert np.all(ae[_abi.ACC_STEPS] > 0)
    for r, a in ((r0, a0), (r1, a1)):
        np.testing.assert_array_equal(a[_abi.ACC_STEPS], ae[_abi.ACC_STEPS])
        np.testing.assert_array_equal(a[_abi.ACC_ON_POST], ae[_abi.ACC_ON_POST])
        np.testing.assert_allclose(r, re, rtol=1e-9, atol=1e-9)


@pytest.mark.parametrize("variant", ["yaw_row_fast", "euler_yaw0"])
@pytest.mark.parametrize("chunks", [[1200], [401, 555, 244]])
def test_rewards_other_fast_flavours_match_step_api(variant, chunks):
    """qt_rollout_rewards on the fast flavours test_rewards_fast_flavour_matches_exact
    does not reach: the staged fast step (a heuristic-LQR gain with a
    yaw-rate row, where the reward comes from sqrt_noscale errors and the
    boundary terms from sqrt_pos) and the Euler closed form of the
    yaw-at-rest flavour; in one launch and in uneven chunks.  Reference: the
    same episodes stepped through the per-step API (BatchedQuadcopterEnv.step_closed,
    its own exact-step kernel), the reward summed per step in order, the last
    post-step error, the step and on-target counts."""
    import torch

    from quadtrack import BatchedQuadcopterEnv, _abi, core
    from quadtrack.controllers import BatchedLQR, BatchedRiccatiLQR
    from quadtrack.rollout import build_batch
    from quadtrack.train import env_config_for

    dev = _abi.require_gpu()
    cfg = env_config_for(7, "circular", 12.0)
    if variant == "euler_yaw0":
        cfg.simulation.integrator = "euler"
        ctl = BatchedRiccatiLQR({"dt": 0.01}, device=dev)
    else:
        K = BatchedLQR({}).gains()[0].cpu().numpy().copy()
        K[3, 0], K[3, 4] = 0.02, -0.01
        ctl = BatchedLQR({"K": K}, device=dev)
    env = cfg.to_params()
    n = 300
    batch = build_batch(ctl, cfg, n, seeds=np.arange(n))
    st = core.RolloutState.empty(n, dev)
    core.reset(env, batch, st)
    reward = torch.zeros(2, n, dtype=torch.float64, device=dev)
    for k in chunks:
        core.rollout_rewards(env, ctl.ctrl, core.criteria(), batch, st, k, reward)
    # the per-step API over the same episodes (freeze_done: the rollout stops at done)
    benv = BatchedQuadcopterEnv(n, cfg)
    benv.reset(np.arange(n))
    total = torch.zeros(n, dtype=torch.float64, device=dev)
    last = torch.zeros(n, dtype=torch.float64, device=dev)
    done_prev = torch.zeros(n, dtype=torch.bool, device=dev)
    for _ in range(sum(chunks)):
        _, r, done, info = benv.step_closed(ctl)
        active = ~done_prev
        total = torch.where(active, total + r, total)
        last = torch.where(active, info["tracking_error"], last)
        done_prev = done.clone()
    np.testing.assert_array_equal(st.acc[_abi.ACC_STEPS].cpu().numpy(), info["step"].cpu().numpy())
    np.testing.assert_array_equal(st.acc[_abi.ACC_ON_POST].cpu().numpy(), info["on_target_count"].cpu().numpy())
    np.testing.assert_allclose(reward[0].cpu().numpy(), total.cpu().numpy(), rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(reward[1].cpu().numpy(), last.cpu().numpy(), rtol=1e-9, atol=1e-9)
