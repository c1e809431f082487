"""wab_gym_amd — MI355X-native batched Wolves-and-Bushes step (hot path of wab-gym).

    from wab_gym_amd import BatchedWolvesAndBushesEnv, default_game_options
    env = BatchedWolvesAndBushesEnv(num_envs=65536, device="cuda:0")
    obs = env.reset()
    obs, reward, done, info = env.step(actions)      # actions: [num_envs] ints

The step runs as one fused HIP kernel for gfx950 behind the C-ABI of include/wab.h
(libwab_hip.so, built in-tree by __graft_entry__.build()).  Importing this package does
not load the library; constructing an env does, and fails loudly if it is missing.
"""
from .options import default_game_options, make_config, bush_thresholds, view_masks  # noqa: F401
from .spaces import Discrete, Box, Tuple, DummySpec  # noqa: F401


def __getattr__(name):
    if name == "BatchedWolvesAndBushesEnv":
        from .env import BatchedWolvesAndBushesEnv

        return BatchedWolvesAndBushesEnv
    if name in ("BatchedWolvesAndBushesEnvEgoCentric", "BatchedWolvesAndBushesEnvEgocentricJustBushes"):
        from . import egocentric

        return getattr(egocentric, name)
    if name == "EpisodeMonitor":
        from .monitor import EpisodeMonitor

        return EpisodeMonitor
    if name == "PragmaticObsWrapper":
        from .wrappers import PragmaticObsWrapper

        return PragmaticObsWrapper
    raise AttributeError(name)


__all__ = ["BatchedWolvesAndBushesEnv", "default_game_options", "make_config", "bush_thresholds"]
