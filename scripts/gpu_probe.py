import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import sys, time, numpy as np, torch
import os; sys_path_root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, 'oracle'); import oracle as O
from f110_gymnasium_ros2_jazzy_amd.sim import BatchSim
from f110_gymnasium_ros2_jazzy_amd.maps import load_map
print(torch.cuda.get_device_name(0), flush=True)
tm = load_map('Spielberg_map')
sim = BatchSim(tm, n_envs=2, n_agents=1, noise_std=0.0, keep_f64_scans=True)
g = np.load('tests/golden/scans_Spielberg_map.npz')
sc, lk, rc = sim.scan_batch(g['poses'], probe=True); torch.cuda.synchronize()
sc = sc.cpu().numpy(); print('probe scans exact', np.array_equal(sc, g['scans']), np.abs(sc-g['scans']).max(), 'lookups', np.array_equal(lk.cpu().numpy(), g['lookups']), 'rc', np.array_equal(rc.cpu().numpy(), g['hit_rc']), flush=True)
sc2 = sim.scan_batch(g['poses']); torch.cuda.synchronize(); sc2=sc2.cpu().numpy()
print('pool scans exact', np.array_equal(sc2, g['scans']), np.abs(sc2-g['scans']).max(), flush=True)
d = np.load('tests/golden/dynamics.npz')
F = sim.dynamics_batch(d['X'], d['U']).cpu().numpy()
print('dyn maxrel', np.max(np.abs(F-d['F'])/np.maximum(np.abs(d['F']),1e-300)), 'exact rows', np.all(F==d['F'],1).sum(), flush=True)
# sim trace 1 agent
t = np.load('tests/golden/sim_1agent_crash.npz')
sim1 = BatchSim(tm, n_envs=1, n_agents=1, noise_std=0.0, keep_f64_scans=True)
st = np.zeros((7,1)); st[0,0],st[1,0],st[4,0] = t['poses'][0]
sim1.set_state(st, np.zeros((2,1)), np.zeros(1,np.int32))
mx=0; exs=0; exsc=0
for k in range(t['actions'].shape[0]):
    out = sim1.step(t['actions'][k][None].astype(np.float32)); torch.cuda.synchronize()
    s = sim1.agent_states().cpu().numpy()[0]
    mx=max(mx, np.abs(s-t['states'][k]).max()); exs += np.array_equal(s, t['states'][k]); exsc += np.array_equal(out.scans_f64.cpu().numpy()[0], t['scans'][k])
print('1agent_crash: state maxabs', mx, 'exact states', exs, 'exact scans', exsc, 'of', t['actions'].shape[0], flush=True)
# throughput probe
E=4096
simb = BatchSim(tm, n_envs=E, n_agents=1, noise_std=0.01, autoreset=True, spawn_poses=__import__('f110_gymnasium_ros2_jazzy_amd').centerline_spawns('Spielberg',1))
poses = torch.as_tensor(__import__('f110_gymnasium_ros2_jazzy_amd').centerline_spawns('Spielberg',1)[:E], device='cuda')
simb.reset(poses)
acts = torch.rand(64, E, 1, 2, device='cuda'); acts[...,0] = acts[...,0]*0.8378-0.4189; acts[...,1]*=20
for i in range(20): simb.step(acts[i%64], minimal_outputs=True)
torch.cuda.synchronize(); simb.reset_counters()
t0=time.time()
for i in range(200): simb.step(acts[i%64], minimal_outputs=True)
torch.cuda.synchronize(); dt=time.time()-t0
lk, rays = simb.read_counters()
print(f'E={E}: {dt/200*1e3:.3f} ms/step, {E*200/dt/1e6:.3f} M env-steps/s, mean lookups/ray {lk/rays:.2f}', flush=True)
