"""Probe: a mesh rock inserted from a URDF file through the ScenarI/O mirror
(prints the base pose and contact count over time)."""
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "gym-ignition_amd", "python"), os.path.join(ROOT, "tests")]
from mesh_models import mesh_body_urdf, rock_vertices, write_obj  # noqa: E402
from mwstep import get_model_file  # noqa: E402
from scenario import core  # noqa: E402
from scenario import gazebo as scenario  # noqa: E402

d = tempfile.mkdtemp()
v, f = rock_vertices(4)
os.makedirs(os.path.join(d, "meshes"))
write_obj(os.path.join(d, "meshes", "rock.obj"), v, f)
mf = os.path.join(d, "rock.urdf")
open(mf, "w").write(mesh_body_urdf("meshes/rock.obj", mass=3.0, half=(0.12, 0.08, 0.06)))
gz = scenario.GazeboSimulator(0.001, 1.0, 1)
assert gz.initialize()
world = gz.get_world().to_gazebo()
assert world.insert_model(get_model_file("ground_plane"))
q = np.array([0.9, 0.3, 0.2, 0.1]) / np.linalg.norm([0.9, 0.3, 0.2, 0.1])
assert world.insert_model(mf, core.Pose([0, 0, 0.3], [float(x) for x in q]), "rock")
rock = world.get_model("rock")
print("links", rock.link_names(), "contacts enabled", rock.enable_contacts(True))
sc = gz._scene
print("scene models", sc.models)
for t in range(2500):
    assert gz.run()
    if t % 250 == 0 or t == 2499:
        print(t, np.round(rock.base_position(), 4), "in_contact", rock.get_link("body").in_contact(),
              "n", len(rock.contacts()), "scene contacts w0", len(sc.contacts(0)))
