"""f110_gym.envs namespace of the reference, backed by libf110 on MI355X."""
from f110_gymnasium_ros2_jazzy_amd.f110_env import F110Env, Integrator  # noqa: F401
