"""Transcribes the ROS tf transforms the reference's author logged from a real
run into tests/golden/tf_log_transforms.json (data only: per transform its
source line, frame ids, stamp, translation (x, y, z) and rotation quaternion
(x, y, z, w), exactly as printed).

Source: /root/reference/scripts/back_up_files/log.txt (`rostopic echo /tf`
output: STag marker poses in the camera frame and the AHRS orientation).  Run
in this container; the fixture travels, the reference does not.  These pin
the quaternion conventions of pose_estimation_module.py:15-65 (tf's
quaternion_matrix and the trace-branch rotation_matrix_to_quaternion) on real
ROS data (tests/test_pose_module.py)."""
import json
import os

SRC = "/root/reference/scripts/back_up_files/log.txt"


def main():
    lines = open(SRC).read().split("\n")
    out = []
    for i, line in enumerate(lines):
        if line.strip() != "translation:":
            continue
        def val(k, key):
            name, v = lines[k].strip().split(":", 1)
            assert name == key, (k, lines[k])
            return float(v)
        t = [val(i + 1, "x"), val(i + 2, "y"), val(i + 3, "z")]
        assert lines[i + 4].strip() == "rotation:"
        q = [val(i + 5, "x"), val(i + 6, "y"), val(i + 7, "z"), val(i + 8, "w")]
        # header fields above the transform: frame_id / child_frame_id / stamp
        j = i
        while not lines[j].strip().startswith("child_frame_id:"):
            j -= 1
        child = lines[j].split(":", 1)[1].strip().strip('"')
        frame = lines[j - 1].split(":", 1)[1].strip().strip('"')
        secs = int(lines[j - 3].split(":", 1)[1])
        nsecs = int(lines[j - 2].split(":", 1)[1])
        out.append({"line": i + 1, "frame_id": frame, "child_frame_id": child, "secs": secs, "nsecs": nsecs,
                    "t": t, "q": q})
    doc = {"source": "scripts/back_up_files/log.txt", "count": len(out), "transforms": out}
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tf_log_transforms.json")
    with open(path, "w") as fh:
        json.dump(doc, fh, indent=0)
    print(path, len(out))


if __name__ == "__main__":
    main()
