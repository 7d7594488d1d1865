"""Insert a shipped model into a world under a unique name."""

from scenario import core as scenario_core

from gym_ignition.utils.scenario import get_unique_model_name


def insert(world, base_name: str, model_file: str, position, orientation):
    name = get_unique_model_name(world, base_name)
    pose = scenario_core.Pose(position, orientation)
    if not world.to_gazebo().insert_model(model_file, pose, name):
        raise RuntimeError("Failed to insert model")
    return world.get_model(name)
