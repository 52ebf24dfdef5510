"""MI355X-native batched F1TENTH simulator (the f110_gym per-step hot path).

Public surface:
  BatchSim        n_envs x n_agents cars on one GPU (sim.py)
  F110Env         drop-in for f110_gym.envs.F110Env (f110_env.py)
  F110VectorEnv   Gymnasium-style vector env (vector_env.py)
  load_map        map yaml + image -> TrackMap with exact EDT (maps.py)
"""
from .maps import TrackMap, load_map, centerline_spawns  # noqa: F401
from ._lib import F110Error, INTEGRATOR_RK4, INTEGRATOR_EULER  # noqa: F401

__version__ = "0.1.0"


def __getattr__(name):  # lazy: torch-backed classes
    if name == "BatchSim":
        from .sim import BatchSim
        return BatchSim
    if name == "F110Env":
        from .f110_env import F110Env
        return F110Env
    if name == "F110VectorEnv":
        from .vector_env import F110VectorEnv
        return F110VectorEnv
    raise AttributeError(name)
