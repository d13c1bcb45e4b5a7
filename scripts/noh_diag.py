import sys, numpy as np
sys.path.insert(0, 'sph-exa_amd/python')
import sphexa_amd as sx
from sphexa_amd import ic
for side in (50, 300):
    arrays, lim, bnd, dt0 = ic.noh(side)
    n = arrays['x'].size
    ctx = sx.Context(0)
    sim = sx.Sim(ctx, n, sx.make_box(lim, bnd))
    sim.set_state(arrays, dt0, dt0)
    e = sim.conserved(); print(side, n, 'e0', {k: e[k] for k in ('ecin','eint','etot')}, flush=True)
    for s in range(3):
        sim.step()
        e = sim.conserved(); st = sim.stats(); sc = sim.scalars()
        f = sim.get(['vx','vy','vz','temp','h','nc','x'])
        v2 = f['vx'].astype(float)**2 + f['vy']**2 + f['vz']**2
        print(' step', s, {k: e[k] for k in ('ecin','eint','etot')}, st, sc, 'v2 mean', v2.mean(), 'temp', f['temp'].min(), f['temp'].max(),
              'h', f['h'].min(), f['h'].max(), 'nc', f['nc'].min(), f['nc'].max(), 'nan', np.isnan(v2).sum(), flush=True)
    sim.close(); ctx.close()
