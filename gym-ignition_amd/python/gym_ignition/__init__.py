"""gym_ignition mirror: Task / Runtime interfaces and the Gazebo runtime,
running on the MI355X stepper through the ``scenario`` mirror."""
