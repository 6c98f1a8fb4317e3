"""dvo_pose_chain_host (rank 0's absolute chain of a sharded stream, include/dvo.h):
T_abs[p] = T_abs[p-1] . T_rel[p] (visual_odometry_v3.py:367) in the device kernel's
arithmetic order, element (r, c) = ((t_r0 A_0c + t_r1 A_1c) + t_r2 A_2c) + t_r3 A_3c,
checked byte for byte against a Python restatement of that order (Python floats are
IEEE doubles, no contraction).  CPU only: the host chain needs no GPU."""
import numpy as np
import pytest


def _chain_py(T_rel, T0):
    t = [float(v) for v in T0.reshape(16)]
    out = np.empty_like(T_rel)
    for p in range(len(T_rel)):
        A = [float(v) for v in T_rel[p].reshape(16)]
        u = [0.0] * 16
        for r in range(4):
            for c in range(4):
                u[r * 4 + c] = ((t[r * 4] * A[c] + t[r * 4 + 1] * A[4 + c]) + t[r * 4 + 2] * A[8 + c]) + \
                    t[r * 4 + 3] * A[12 + c]
        t = u
        out[p] = np.array(t).reshape(4, 4)
    return out, np.array(t)


@pytest.mark.parametrize("n", [0, 1, 7, 300])
def test_host_chain_matches_restated_order(n):
    from droplet_visual_odometry_amd import _native
    from droplet_visual_odometry_amd import transformations as tr
    lib = _native.load_library()
    rng = np.random.default_rng(n + 5)
    T_rel = np.zeros((max(n, 1), 4, 4))
    for p in range(n):
        T = tr.euler_matrix(*rng.uniform(-0.3, 0.3, 3))
        T[:3, 3] = rng.uniform(-0.5, 0.5, 3)
        T_rel[p] = T
    T0 = tr.euler_matrix(0.1, -0.2, 0.3)
    T0[:3, 3] = (1.0, -2.0, 0.5)
    want, want_carry = _chain_py(T_rel[:n], T0)
    carry = np.ascontiguousarray(T0.reshape(16)).copy()
    out = np.zeros((max(n, 1), 4, 4))
    assert lib.dvo_pose_chain_host(T_rel.ctypes.data, n, carry.ctypes.data, out.ctypes.data) == 0
    assert out[:n].tobytes() == want.tobytes()
    assert carry.tobytes() == (want_carry.tobytes() if n else T0.reshape(16).tobytes())


def test_host_chain_rejects_null_arguments():
    from droplet_visual_odometry_amd import _native
    lib = _native.load_library()
    assert lib.dvo_pose_chain_host(None, 3, None, None) != 0
    assert lib.dvo_pose_chain_host(None, -1, None, None) != 0
    assert lib.dvo_pose_chain_host(None, 0, None, None) == 0  # empty chain: nothing read or written
