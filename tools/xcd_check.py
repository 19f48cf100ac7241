"""Bitwise check: the per-XCD LPT orders (knob xcd_lpt 1) against the global LPT order (0) at cfg 3."""
import sys, torch
sys.path.insert(0, ".")
from bench import CONFIGS
from gaussian_splatting_lightning_amd import _native
from gaussian_splatting_lightning_amd.rasterizer import GaussianRasterizationSettings, backward_raw, forward_raw
from gaussian_splatting_lightning_amd.synthetic import make_camera, make_scene, make_upstream
cfg = CONFIGS["cfg3"]; dev = torch.device("cuda", 0)
sc = make_scene(cfg["n"], cfg["deg"], seed=0, stress_fraction=cfg["stress"]).to(dev)
cam = make_camera(cfg["W"], cfg["H"]).to(dev)
dc, di = (t.to(dev) for t in make_upstream(cfg["W"], cfg["H"], 0))
rs = GaussianRasterizationSettings(cfg["H"], cfg["W"], cam.tanfovx, cam.tanfovy, torch.zeros(3, device=dev), 1.0,
                                   cam.viewmatrix, cam.projmatrix, cfg["deg"], cam.campos, False, False, False)
out = {}
for v in (0, 1):
    _native.set_tuning("xcd_lpt", v)
    c, r, i, st = forward_raw(sc.means3D, sc.shs, None, sc.opacities, sc.scales, sc.rotations, None, rs)
    g = backward_raw(st, rs, dc, di)
    torch.cuda.synchronize()
    out[v] = [c.clone(), i.clone()] + [t.clone() for t in g if isinstance(t, torch.Tensor)]
for v in (1,):
    same = all(torch.equal(a, b) for a, b in zip(out[0], out[v]))
    print("xcd_lpt", v, "bitwise equal to default:", same, flush=True)
    assert same
