import sys, numpy as np, torch
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/tests'); sys.path.insert(0, '/root/repo/oracle')
import oracle; oracle.build()
from conftest import synth_frames
from droplet_visual_odometry_amd.stream import FrameStream
from droplet_visual_odometry_amd import ops
frames, K = synth_frames(640, 480, range(4))
fs = FrameStream(640, 480, K, nfeatures=1000, max_frames=4)
rec = fs.process(torch.from_numpy(frames).cuda()); fs.sync()
recs = FrameStream.records_numpy(rec, 3)
kp = None
for i in range(3):
    ref = oracle.pair_pose(frames[i], frames[i+1], K, 1000, kp_prev=kp); kp = (ref['kp_cur'], ref['desc_cur'])
    r = recs[i]
    print(i, 'iters', r['ransac_iters'], ref['iters'], 'hyps', r['n_hypotheses'], 'inl', r['n_inliers'], int(ref['mask'].sum()),
          'E equal', np.array_equal(r['E'].reshape(3,3), ref['E']), 'm', len(ref['q']))
    E, mask = ops.find_essential_mat(ref['p1'], ref['p2'], K)
    print('   per-call E equal', np.array_equal(E, ref['E']), int(mask.sum()))
    for mi in (10, 26, 35, 64, 65, 100):
        Eo, mo, io = oracle.find_essential(ref['p1'], ref['p2'], K, max_iters=mi)
        Eg, mg = ops.find_essential_mat(ref['p1'], ref['p2'], K, max_iters=mi)
        print('   max_iters', mi, 'oracle iters', io, 'E eq', np.array_equal(Eg, Eo), int(mo.sum()), int(mg.sum()))
