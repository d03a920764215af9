"""Compare one golden fixture step across kernel layouts (GPU debugging aid)."""
import sys
import numpy as np
import torch
sys.path[:0] = ['.', 'tests', 'swarmacb-isaaclab_amd']
import parity
from oracle import oracle as O
from SwarmACB_isaac.engine import SwarmEngine

name = sys.argv[1] if len(sys.argv) > 1 else "isaac_dgt_cyclamen_mid"
fx = parity.load(name)
env, meta = O.fixture_env(fx)
dev = torch.device("cuda:0")
before, kw = O.fixture_step_inputs(fx, 0)
state = {k[len("before_"):]: v for k, v in before.items()}
d = kw["draws"]
res = {}
for layout in (4, 103):
    eng = SwarmEngine(meta["mission"], meta["profile"], env.E, env.N, env.obs_dim, meta["discrete"], env.cfg.max_len,
                      1, 0, 0, dev, layout=layout)
    eng.reset()
    eng.load_state(state)
    rp = {"rab_uniform": torch.as_tensor(d["rab_u_obs"][None].copy()).to(dev),
          "turn_steps": torch.as_tensor(d["turns"][None].astype(np.int32)).to(dev),
          "spawn_uniform": torch.as_tensor(np.ascontiguousarray(d["spawn_u"])).to(dev), "spawn_draws": d["spawn_k"],
          "spawn_yaw_uniform": torch.as_tensor(np.ascontiguousarray(d["spawn_yaw_u"])).to(dev)}
    a = torch.as_tensor(np.ascontiguousarray(kw["actions"])).to(dev)
    a = a.to(torch.int32) if meta["discrete"] else a.float()
    obs, rew, tr = eng.step(a.contiguous(), 1, replay=rp)
    res[layout] = (obs.cpu().numpy(), eng.dump_state())
    eng.close()
ref = parity.reference_after(fx, 0)
for layout, (obs, st) in res.items():
    print("layout", layout, "obs max err", np.abs(obs - ref["obs"]).max(), "pos err", np.abs(st["pos"] - ref["pos"]).max(),
          "cache err", np.abs(st["cache"] - ref["cache"]).max())
o1, o3 = res[1][0], res[103][0]
bad = np.argwhere(np.abs(o1 - o3) > 1e-5)
print("first diffs (env, robot, ch):", bad[:12].tolist())
for e, i, c in bad[:6]:
    print(e, i, c, "L1", o1[e, i, c], "L103", o3[e, i, c], "ref", ref["obs"][e, i, c])
