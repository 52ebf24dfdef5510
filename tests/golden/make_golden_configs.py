"""Reward configurations of tests/golden/reward.npz (shared by make_golden.py and the tests)."""

REWARD_CONFIGS = {
    # rl_training/train_ddpg.py:125-146
    "train_ddpg": dict(w_prog=5.0, alive_bonus=0.5, grace_steps_wall=25, grace_steps_opp=175, w_lat=0.25,
                       lat_cap=3.0, near_wall_dist=0.30 / 30, w_wall=0.30, wall_quantile=0.10, opp_safe_dist=0.60,
                       w_opp=0.30, w_rel_lead=0.0),
    # every term early: short grace periods, lead shaping, wide bubbles
    "all_terms": dict(w_prog=1.2, alive_bonus=0.02, grace_steps_wall=3, grace_steps_opp=3, w_lat=0.35, lat_cap=4.0,
                      near_wall_dist=0.12, w_wall=1.0, wall_quantile=0.05, opp_safe_dist=3.0, w_opp=0.8,
                      w_rel_lead=0.3, lead_clip=0.5, forward_sign=-1.0),
}
