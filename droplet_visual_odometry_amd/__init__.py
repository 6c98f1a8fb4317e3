"""droplet_visual_odometry_amd — MI355X-native visual-odometry front end.

The hot path of theivyzhang/droplet_visual_odometry (ORB detect -> Hamming
match -> findEssentialMat/RANSAC -> recoverPose, scripts/visual_odometry_v3.py
and scripts/pose_estimation_module.py) as hand-written HIP kernels for gfx950
behind a C ABI (include/dvo.h), with:

  cv          the cv2 operator surface the reference calls (GPU-backed)
  ops         numpy-level wrappers of the per-call C-ABI entry points
  stream      batched device-resident frame streams (many pairs per launch)
  dist        frame sharding across GPUs + RCCL all-gather of pose records
  dropin/     visual_odometry_v3.py / pose_estimation_module.py drop-ins
  synth       seeded synthetic frame streams for tests and bench.py
"""
import os as _os

DROPIN_DIR = _os.path.join(_os.path.dirname(_os.path.abspath(__file__)), "dropin")
__version__ = "0.1.0"
