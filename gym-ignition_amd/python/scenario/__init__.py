"""ScenarI/O mirror over the MI355X stepper.

``from scenario import core, gazebo`` works as with the reference's SWIG
bindings (``/root/reference/bindings/__init__.py``); the simulator behind
``gazebo.GazeboSimulator`` is the native many-worlds library, not ign-gazebo.
"""

from . import core, gazebo  # noqa: F401
