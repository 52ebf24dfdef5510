"""Drop-in package name of the reference (f110_gymnasium/gym/f110_gym).

``gym.make('f110_gym:f110-v0', ...)`` resolves here: the id is registered
with gymnasium (when installed) and points at the MI355X-backed F110Env.
"""
try:
    from gymnasium.envs.registration import register, registry

    if "f110-v0" not in registry:
        register(id="f110-v0", entry_point="f110_gym.envs:F110Env")
except Exception:  # gymnasium absent: import f110_gym.envs.F110Env directly
    pass
