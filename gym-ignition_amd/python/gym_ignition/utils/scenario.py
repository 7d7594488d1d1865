"""Name helpers used by the runtimes and model wrappers
(reference: python/gym_ignition/utils/scenario.py:13-58)."""

import itertools

_worlds_seen = set()


def _first_free(base: str, taken) -> str:
    for k in itertools.count():
        candidate = base if k == 0 else f"{base}{k}"
        if candidate not in taken:
            return candidate


def get_unique_model_name(world, model_name: str) -> str:
    """`cartpole`, `cartpole1`, `cartpole2`, ... : the first name not in the world."""
    return _first_free(model_name, set(world.model_names()))


def get_unique_world_name(world_name: str) -> str:
    """Unique across the process (the reference asks the ECM singleton)."""
    name = _first_free(world_name, _worlds_seen)
    _worlds_seen.add(name)
    return name
