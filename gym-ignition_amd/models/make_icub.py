"""Generate icub.urdf: an iCub-class floating-base humanoid with the reference
wrapper's joint names, counts and initial posture, for BASELINE config 5
(the reference's iCub model package, gym_ignition_models' iCubGazeboV2_5, is
not available offline, so this is an authored stand-in, not iCub's
parameters).

What the reference pins (python/gym_ignition_environments/models/icub.py):
  * DOFS = 32, NUM_JOINTS = 32, NUM_LINKS = 39 (:15-17);
  * the 32 joint names and the initial posture (:19-40): bent knees
    (-1.05), hip pitch 0.48, ankle pitch -0.57, torso pitch 0.1, arms
    abducted (shoulder roll 0.435) with the elbows at 0.54;
  * the insertion pose (0, 0, 0.572), orientation wxyz (0, 0, 0, 1) (:86).
This model has exactly those 32 revolute joints and 39 links: the 33 moving
bodies (root_link + one per joint) plus six force/torque-sensor frames
welded by fixed joints as on the iCub (l/r_leg_ft_sensor between hip roll
and hip yaw, l/r_foot_ft_sensor under the ankle, l/r_arm_ft_sensor between
shoulder yaw and elbow), kept as links with
<gazebo reference><preserveFixedJoint> (sdformat's switch; the physics lumps
their inertia into the parent body either way).  Link names follow the iCub's
(root_link, torso_1, torso_2, chest, neck_1, neck_2, head, l_shoulder_1..3,
l_upper_arm, l_elbow_1, l_forearm, l_wrist_1, l_hand, l_hip_1..3,
l_upper_leg, l_lower_leg, l_ankle_1, l_ankle_2, l_foot, and r_*).

Geometry: iCub-like round numbers (30.7 kg; thigh 0.2236 m, shank 0.213 m,
hip joints 0.12 m below the pelvis frame, sole 0.07 m below the ankle), so
that at the wrapper's posture and pose the soles hang 4 mm above the ground
and the robot settles onto its feet.  The root_link frame points backward
(x) as the iCub's does; the wrapper's orientation (a half turn about z) makes
the robot face world +x.  Collision: one box per foot (8 contact corners
each).  Tree depth 10 (root -> torso x3 -> shoulder x3 -> elbow -> wrist x3).

    python make_icub.py > icub.urdf
"""

import math

# the reference wrapper's posture (icub.py:19-40), here in the URDF's joint order
INITIAL_POSITIONS = {
    "l_knee": -1.05, "l_ankle_pitch": -0.57, "l_ankle_roll": -0.024,
    "l_hip_pitch": 0.48, "l_hip_roll": 0.023, "l_hip_yaw": -0.005,
    "l_elbow": 0.54, "l_wrist_pitch": 0.0, "l_wrist_prosup": 0.0, "l_wrist_yaw": 0.0,
    "l_shoulder_pitch": -0.159, "l_shoulder_roll": 0.435, "l_shoulder_yaw": 0.183,
    "neck_pitch": 0.0, "neck_roll": 0.0, "neck_yaw": 0.0,
    "r_knee": -1.05, "r_ankle_pitch": -0.57, "r_ankle_roll": -0.024,
    "r_hip_pitch": 0.48, "r_hip_roll": 0.023, "r_hip_yaw": -0.005,
    "r_elbow": 0.54, "r_wrist_pitch": 0.0, "r_wrist_prosup": 0.0, "r_wrist_yaw": 0.0,
    "r_shoulder_pitch": -0.159, "r_shoulder_roll": 0.435, "r_shoulder_yaw": 0.183,
    "torso_pitch": 0.1, "torso_roll": 0.0, "torso_yaw": 0.0,
}

THIGH, SHANK, HIP_DROP, SOLE = 0.2236, 0.213, 0.12, 0.07
FOOT = (0.16, 0.07, 0.02)            # sole box (length x width x height)
FOOT_X = -0.037                      # box centre along root x (backward): 3.7 cm in front of the ankle
FOOT_Y = 0.016                       # ... and 1.6 cm outward: the centre of pressure of the held posture


def box_inertia(m, x, y, z):
    return m / 12 * (y * y + z * z), m / 12 * (x * x + z * z), m / 12 * (x * x + y * y)


def rod_inertia(m, length, r=0.03):
    i = m * (3 * r * r + length * length) / 12
    return i, i, m * r * r / 2


def link(name, mass, com=(0, 0, 0), inertia=None, collision=""):
    ixx, iyy, izz = inertia or (1e-3, 1e-3, 1e-3)
    return (f'  <link name="{name}">\n    <inertial>\n      <origin xyz="{com[0]:.4f} {com[1]:.4f} {com[2]:.4f}" '
            f'rpy="0 0 0"/>\n      <mass value="{mass}"/>\n      <inertia ixx="{ixx:.6g}" ixy="0" ixz="0" '
            f'iyy="{iyy:.6g}" iyz="0" izz="{izz:.6g}"/>\n    </inertial>\n{collision}  </link>\n')


def joint(name, parent, child, axis, xyz=(0, 0, 0), lower=-1.5, upper=1.5, effort=80.0):
    return (f'  <joint name="{name}" type="revolute">\n    <parent link="{parent}"/>\n    <child link="{child}"/>\n'
            f'    <origin xyz="{xyz[0]:.4f} {xyz[1]:.4f} {xyz[2]:.4f}" rpy="0 0 0"/>\n    <axis xyz="{axis}"/>\n'
            f'    <limit lower="{lower}" upper="{upper}" effort="{effort}" velocity="10"/>\n  </joint>\n')


def ft_sensor(name, parent, child, xyz=(0, 0, 0)):
    """A welded force/torque-sensor frame: fixed joint kept by sdformat."""
    return (f'  <joint name="{name}" type="fixed">\n    <parent link="{parent}"/>\n    <child link="{child}"/>\n'
            f'    <origin xyz="{xyz[0]:.4f} {xyz[1]:.4f} {xyz[2]:.4f}" rpy="0 0 0"/>\n  </joint>\n'
            f'  <gazebo reference="{name}">\n    <preserveFixedJoint>true</preserveFixedJoint>\n  </gazebo>\n')


# axes in the root_link frame (x backward, y to the robot's right, z up):
# positive hip pitch / elbow swing the limb forward (-x), negative knee folds
# the shank back, negative ankle pitch tilts the sole back level
PITCH_FWD, PITCH_BACK, ROLL, YAW = "0 1 0", "0 -1 0", "1 0 0", "0 0 1"


def main():
    out = ['<?xml version="1.0"?>\n<!-- generated by make_icub.py: an iCub-class 32-dof floating-base humanoid '
           'with the gym-ignition iCub wrapper\'s joint names, 39 links (see the script for provenance) -->\n'
           '<robot name="iCubGazeboV2_5">\n']
    out.append(link("root_link", 4.0, inertia=box_inertia(4.0, 0.1, 0.2, 0.12)))
    # torso: root -> torso_1 -> torso_2 -> chest (torso pitch leans forward)
    out.append(joint("torso_pitch", "root_link", "torso_1", PITCH_BACK, (0, 0, 0.06), -0.4, 1.4))
    out.append(link("torso_1", 0.5))
    out.append(joint("torso_roll", "torso_1", "torso_2", ROLL, (0, 0, 0), -0.5, 0.5))
    out.append(link("torso_2", 0.5))
    out.append(joint("torso_yaw", "torso_2", "chest", YAW, (0, 0, 0), -0.9, 0.9))
    out.append(link("chest", 6.0, (0.01, 0, 0.14), box_inertia(6.0, 0.15, 0.26, 0.28)))
    # neck -> head
    out.append(joint("neck_pitch", "chest", "neck_1", PITCH_BACK, (0, 0, 0.30), -0.9, 0.9, 20.0))
    out.append(link("neck_1", 0.2))
    out.append(joint("neck_roll", "neck_1", "neck_2", ROLL, (0, 0, 0), -0.6, 0.6, 20.0))
    out.append(link("neck_2", 0.2))
    out.append(joint("neck_yaw", "neck_2", "head", YAW, (0, 0, 0), -0.9, 0.9, 20.0))
    out.append(link("head", 1.8, (0, 0, 0.09), box_inertia(1.8, 0.14, 0.14, 0.16)))
    # arms: left at -y (the robot's left), roll axis signed so +roll abducts
    for side, s in (("l", -1.0), ("r", 1.0)):
        roll = "-1 0 0" if s < 0 else ROLL
        out.append(joint(f"{side}_shoulder_pitch", "chest", f"{side}_shoulder_1", PITCH_BACK, (0, s * 0.11, 0.26),
                         -1.7, 0.6, 40.0))
        out.append(link(f"{side}_shoulder_1", 0.3))
        out.append(joint(f"{side}_shoulder_roll", f"{side}_shoulder_1", f"{side}_shoulder_2", roll, (0, 0, 0),
                         0.0, 2.8, 40.0))
        out.append(link(f"{side}_shoulder_2", 0.3))
        out.append(joint(f"{side}_shoulder_yaw", f"{side}_shoulder_2", f"{side}_shoulder_3", YAW, (0, 0, 0),
                         -0.6, 1.4, 30.0))
        out.append(link(f"{side}_shoulder_3", 0.3, (0, 0, -0.03)))
        out.append(ft_sensor(f"{side}_arm_ft_sensor", f"{side}_shoulder_3", f"{side}_upper_arm", (0, 0, -0.06)))
        out.append(link(f"{side}_upper_arm", 0.9, (0, 0, -0.05), rod_inertia(0.9, 0.15)))
        out.append(joint(f"{side}_elbow", f"{side}_upper_arm", f"{side}_elbow_1", PITCH_FWD, (0, 0, -0.10),
                         0.1, 1.85, 30.0))
        out.append(link(f"{side}_elbow_1", 0.3))
        out.append(joint(f"{side}_wrist_prosup", f"{side}_elbow_1", f"{side}_forearm", YAW, (0, 0, 0), -1.0, 1.0,
                         10.0))
        out.append(link(f"{side}_forearm", 0.6, (0, 0, -0.07), rod_inertia(0.6, 0.14)))
        out.append(joint(f"{side}_wrist_pitch", f"{side}_forearm", f"{side}_wrist_1", PITCH_FWD, (0, 0, -0.14),
                         -1.1, 0.4, 10.0))
        out.append(link(f"{side}_wrist_1", 0.1))
        out.append(joint(f"{side}_wrist_yaw", f"{side}_wrist_1", f"{side}_hand", ROLL, (0, 0, 0), -0.4, 0.4, 10.0))
        out.append(link(f"{side}_hand", 0.3, (0, 0, -0.05), (1.2e-3, 1.2e-3, 6e-4)))
    # legs: hip pitch / roll, the leg F/T sensor, hip yaw, knee, ankle pitch /
    # roll, the foot F/T sensor and the sole
    for side, s in (("l", -1.0), ("r", 1.0)):
        foot = (f'    <collision>\n      <origin xyz="{FOOT_X} {s * FOOT_Y} {-FOOT[2] / 2:.3f}" rpy="0 0 0"/>\n'
                f'      <geometry><box size="{FOOT[0]} {FOOT[1]} {FOOT[2]}"/></geometry>\n    </collision>\n')
        roll = "-1 0 0" if s < 0 else ROLL
        out.append(joint(f"{side}_hip_pitch", "root_link", f"{side}_hip_1", PITCH_FWD, (0, s * 0.07, -HIP_DROP),
                         -0.7, 2.0))
        out.append(link(f"{side}_hip_1", 0.75))
        out.append(joint(f"{side}_hip_roll", f"{side}_hip_1", f"{side}_hip_2", roll, (0, 0, 0), -0.3, 1.5))
        out.append(link(f"{side}_hip_2", 0.8))
        out.append(ft_sensor(f"{side}_leg_ft_sensor", f"{side}_hip_2", f"{side}_hip_3", (0, 0, -0.03)))
        out.append(link(f"{side}_hip_3", 0.3))
        out.append(joint(f"{side}_hip_yaw", f"{side}_hip_3", f"{side}_upper_leg", YAW, (0, 0, 0.03), -1.3, 1.3))
        out.append(link(f"{side}_upper_leg", 1.5, (0, 0, -THIGH / 2), rod_inertia(1.5, THIGH, 0.045)))
        out.append(joint(f"{side}_knee", f"{side}_upper_leg", f"{side}_lower_leg", PITCH_FWD, (0, 0, -THIGH),
                         -2.0, 0.0))
        out.append(link(f"{side}_lower_leg", 1.0, (0, 0, -SHANK / 2), rod_inertia(1.0, SHANK, 0.04)))
        out.append(joint(f"{side}_ankle_pitch", f"{side}_lower_leg", f"{side}_ankle_1", PITCH_BACK, (0, 0, -SHANK),
                         -0.8, 0.6))
        out.append(link(f"{side}_ankle_1", 0.4))
        out.append(joint(f"{side}_ankle_roll", f"{side}_ankle_1", f"{side}_ankle_2", roll, (0, 0, 0), -0.4, 0.4))
        out.append(link(f"{side}_ankle_2", 0.3))
        out.append(ft_sensor(f"{side}_foot_ft_sensor", f"{side}_ankle_2", f"{side}_foot", (0, 0, -SOLE + FOOT[2])))
        out.append(link(f"{side}_foot", 0.6, (FOOT_X, s * FOOT_Y, -FOOT[2] / 2), box_inertia(0.6, *FOOT), foot))
    out.append("</robot>\n")
    return "".join(out)


def sole_height(z_base=0.572):
    """Height of the soles above the ground at the wrapper's posture and pose
    (sagittal chain; the hip / ankle roll offsets are below 1e-4 m)."""
    q = INITIAL_POSITIONS
    drop = (HIP_DROP + THIGH * math.cos(q["l_hip_pitch"]) + SHANK * math.cos(q["l_hip_pitch"] + q["l_knee"])
            + SOLE)
    return z_base - drop


if __name__ == "__main__":
    print(main(), end="")
