"""Oracle pins: the reference's one recorded output plus known-answer tests."""
import math

import pytest
import torch
import torch.nn.functional as F

from oracle import pathtracer_ref as R
from oracle import recipes


def test_reference_checksum():
    """the only run of the reference, reproduced bit for bit."""
    torch.set_num_threads(8)
    out = recipes.baseline_checksum_render()
    assert out.shape == (64, 64, 4)
    assert out.abs().sum().item() == recipes.BASELINE_ABS_SUM


def test_unit_sphere_march_kat():
    """KAT 1: SPHERE_SDF from z=1.5 along -z hits at t=0.5; normal = p_hat; p offset 5e-3."""
    shape = R.MarchedSDF(sdf=R.unit_sphere_sdf, max_steps=16)
    rays = torch.tensor([[0.0, 0.0, 1.5, 0.0, 0.0, -1.0],
                         [0.3, 0.0, 1.5, 0.0, 0.0, -1.0],
                         [0.0, 3.0, 1.5, 0.0, 0.0, -1.0]])
    it, hit = shape.intersect(rays, primary=False)
    assert hit.tolist() == [True, True, False]
    assert abs(it.t[0].item() - 0.5) < 1e-6
    n = it.n[1]
    p_surface = torch.tensor([0.3, 0.0, math.sqrt(1 - 0.09)])
    assert torch.allclose(n, p_surface, atol=1e-3)
    assert torch.allclose(it.p[0], torch.tensor([0.0, 0.0, 1.0 + 5e-3]), atol=1e-5)


def test_zero_init_mlp_is_zero():
    """KAT 2: zero_init SkipConnMLP returns exactly 0; one-sphere blob reduces to |p|-r."""
    torch.manual_seed(0)
    m = R.SkipMLP(num_layers=8, hidden_size=128, in_size=3, out=1, freqs=32,
                  activation="softplus", zero_init=True)
    x = torch.randn(17, 3)
    assert (m(x) == 0).all()
    blob = R.SphereBlobSDF(n=1)
    with torch.no_grad():
        blob.centers.zero_()
        blob.radii.fill_(0.5)
    p = torch.randn(9, 3)
    expect = -torch.log(torch.exp(-32 * (p.norm(dim=-1) - 0.5)).clamp(min=1e-4)) / 32
    assert torch.allclose(blob(p), expect, atol=1e-6)


def test_fourier_encode_kat():
    """KAT 3: e_k through an identity basis gives analytic sin/cos."""
    basis = torch.eye(3)
    x = torch.eye(3)
    enc = R.fourier_encode(x, basis)
    assert torch.allclose(enc[:, 3:6], torch.eye(3) * math.sin(1.0))
    assert torch.allclose(enc[:, 6:9], torch.ones(3, 3) - torch.eye(3) * (1 - math.cos(1.0)))


def test_compositing_closed_form():
    """KAT 4: NeRFLE rolled-cumprod weights with constant sigma (nerf.py:206-213)."""
    S = 8
    ts = torch.linspace(0, 2, S)
    sigma = 0.7
    alpha = 1 - torch.exp(-sigma * ts)
    cp = torch.cumprod((1 - alpha).clamp(min=1e-10), 0)
    cp = torch.roll(cp, 1, 0)
    cp[-1] = 1
    w = alpha * cp
    trans_all = torch.prod(1 - alpha)
    assert torch.isclose(w[0], alpha[0] * trans_all)
    for k in range(1, S - 1):
        assert torch.isclose(w[k], alpha[k] * torch.prod(1 - alpha[:k]))
    assert torch.isclose(w[-1], alpha[-1])


def test_frame_kat():
    """KAT 5: coordinate_system(z) = diag(1,-1,1) (t = s x n flips y, interaction.py:25);
    to_local(from_local(v)) = v_hat."""
    f = R.shading_frame(torch.tensor([[0.0, 0.0, 1.0]]))
    assert torch.allclose(f[0], torch.diag(torch.tensor([1.0, -1.0, 1.0])), atol=1e-6)
    torch.manual_seed(1)
    n = F.normalize(torch.randn(64, 3), dim=-1)
    v = torch.randn(64, 3)
    fr = R.shading_frame(n)
    back = R.frame_to_local(fr, R.frame_from_local(fr, v))
    assert torch.allclose(back, F.normalize(v, dim=-1), atol=1e-5)


def test_rusinkiewicz_kat():
    """KAT 6: param_rusin2(z, z): H = z, phi_d from nz(1e-7) pairs."""
    z = torch.tensor([[0.0, 0.0, 1.0]])
    out = R.rusinkiewicz(z, z)
    # diff = rotate(z about y by c=1, s=-sqrt(1e-6)) = [s, 0, c] normalised -> [-1e-3, 0, 1]
    s = -math.sqrt(1e-6)
    dx = s / math.sqrt(1 + s * s)
    expect_phi = math.cos(math.atan2(1e-7, dx))
    assert abs(out[0, 1].item() - 1.0) < 1e-6
    assert abs(out[0, 0].item() - expect_phi) < 1e-5
    assert abs(out[0, 2].item() - 1 / math.sqrt(1 + s * s)) < 1e-6


def test_point_light_falloff_kat():
    """KAT 7: PointLights falloff scale*normalize(I)/(c + l d + q d^2)."""
    light = R.PointLightRef(location=(0.0, 2.0, 0.0), scale=100.0)
    it = R.Interaction(p=torch.zeros(1, 1, 1, 1, 3))
    ds, le = light.sample_direction(it, torch.ones(1, 1, 1, 1, dtype=torch.bool))
    fall = 1e-6 + 1e-6 * 2 + 1 * 4
    assert torch.allclose(le.reshape(3), torch.full((3,), 100 / math.sqrt(3) / fall), rtol=1e-6)
    assert torch.allclose(ds.d.reshape(3), torch.tensor([0.0, 1.0, 0.0]))


def test_coarse_scan_argmin_kat():
    """KAT 8: the scan's argmin on SPHERE_SDF with a fixed jitter."""
    shape = R.MarchedSDF(sdf=R.unit_sphere_sdf)
    o = torch.tensor([[0.0, 0.0, 2.0]])
    d = torch.tensor([[0.0, 0.0, -1.0]])
    thr, best = shape.coarse_scan(o, d, jitter=0.5)
    step = (2.2 + 0.5 * 2 / 128) / 128
    # |2 - t| - 1 is minimised at the sample closest to t = 2 (the centre)
    k = round(2.0 / step)
    assert abs(best[0, 2].item() - (2.0 - k * step)) < 1e-5
    assert thr.item() < -0.99


def test_fov_camera_kat():
    """FoVCameraRef (renderer/cameras.py:539-575): the unprojected point of NDC (x, y, 1) lies on
    the far plane, so r_d = normalize(C + zfar (f + x tan(fov/2) a right + y tan(fov/2) up)) --
    the point normalised, not the point minus the centre C (:570).  Centre and corner pixels."""
    Rm, Tm = R.look_at_view_transform_ref(dist=2.0, elev=30.0, azim=45.0)
    cam = R.FoVCameraRef(Rm, Tm, znear=1.0, zfar=100.0, fov=60.0)
    C = cam.center()[0]
    el, az = math.radians(30.0), math.radians(45.0)
    want_c = 2.0 * torch.tensor([math.cos(el) * math.sin(az), math.sin(el), math.cos(el) * math.cos(az)])
    assert torch.allclose(C, want_c, atol=1e-6)
    # camera axes are the columns of R: x (right), y (up), z (forward, towards the origin)
    xa, ya, za = Rm[0, :, 0], Rm[0, :, 1], Rm[0, :, 2]
    assert torch.allclose(za, F.normalize(-C, dim=0), atol=1e-6)
    size = 64
    tan = math.tan(math.radians(30.0))
    pos = torch.tensor([[[size / 2, size / 2], [0.0, 0.0]]])  # [W=1, H=2, 2]: centre, corner
    rays = cam.sample_positions(pos, size)
    for j, (nx, ny) in enumerate([(0.0, 0.0), (1.0, 1.0)]):
        far = C + 100.0 * (za + nx * tan * xa + ny * tan * ya)
        assert torch.allclose(rays[0, 0, j, 0, 3:], F.normalize(far, dim=0), atol=2e-6)
        assert torch.allclose(rays[0, 0, j, 0, :3], C, atol=1e-6)


def test_product_look_at_matches_oracle():
    """Host-side camera math of the product (look_at_view_transform, camera centre, inverse full
    projection) equals the oracle's bit for bit: both are the reference's float32 op order."""
    from neural_raytracing_amd.pathtracer.cameras import OpenGLPerspectiveCameras, look_at_view_transform
    for dist, elev, azim in [(1.0, 30.0, 45.0), (2.5, -10.0, 170.0), (1.0, 89.0, 0.0)]:
        Rp, Tp = look_at_view_transform(dist=dist, elev=elev, azim=azim)
        Ro, To = R.look_at_view_transform_ref(dist=dist, elev=elev, azim=azim)
        assert torch.equal(Rp, Ro) and torch.equal(Tp, To)
        cam = OpenGLPerspectiveCameras(R=Rp, T=Tp)
        ref = R.FoVCameraRef(Ro, To, znear=1.0, zfar=100.0)
        assert torch.equal(cam.get_camera_center(), ref.center())
        assert torch.equal(cam.inverse_full_projection(), ref.inverse_full_projection())


def test_plain_nerf_zero_mlps_kat():
    """PlainNeRF (nerf.py:46-74) with zero-initialised MLPs: rgb = tanh(0) = 0, so every ray
    composites to (0 + 1) / 2 = 0.5 whatever the weights of the compositing."""
    torch.manual_seed(0)
    ref = R.PlainNeRFRef(steps=9)
    for m in (ref.first, ref.second):
        for lin in [m.init, *m.layers, m.out]:
            torch.nn.init.zeros_(lin.weight)
            torch.nn.init.zeros_(lin.bias)
    ref.assign_latent(torch.randn(2, 32))
    rays = torch.cat([torch.zeros(2, 3, 4, 1, 3), F.normalize(torch.randn(2, 3, 4, 1, 3), dim=-1)], -1)
    out = ref(rays, None, jitter=0.5, noise=torch.rand(9, 2, 3, 4, 1, 1))
    assert out.shape == (2, 3, 4, 1, 3)
    assert torch.equal(out, torch.full_like(out, 0.5))


def test_plain_nerf_composite_closed_form():
    """PlainNeRF compositing with a constant density: first MLP out bias alpha_raw = c, no noise,
    second MLP out bias b (rgb = tanh(b)): w_0 = a_0 prod(1 - a), w_s = a_s prod_{j<s}(1 - a_j),
    w_{S-1} = a_{S-1}, a_s = 1 - exp(-c t_s) (nerf.py:67-73, the NeRFLE roll quirk)."""
    torch.manual_seed(1)
    S, c, b = 5, 0.7, 0.3
    ref = R.PlainNeRFRef(steps=S)
    for m in (ref.first, ref.second):
        for lin in [m.init, *m.layers, m.out]:
            torch.nn.init.zeros_(lin.weight)
            torch.nn.init.zeros_(lin.bias)
    with torch.no_grad():
        ref.first.out.bias[0] = c
        ref.second.out.bias.fill_(b)
    ref.assign_latent(torch.zeros(1, 32))
    rays = torch.tensor([[0.0, 0.0, 0.0, 0.0, 0.0, -1.0]]).reshape(1, 1, 1, 1, 6)
    out = ref(rays, None, jitter=0.0, noise=torch.zeros(S, 1, 1, 1, 1, 1))
    ts = torch.linspace(0.4, 2.0, S).double()
    a = 1 - torch.exp(-c * ts)
    q = (1 - a).clamp(min=1e-10)
    w = [a[0] * q.prod()] + [a[s] * q[:s].prod() for s in range(1, S - 1)] + [a[S - 1]]
    want = (sum(w) * math.tanh(b) + 1) / 2
    assert abs(out.reshape(-1)[0].item() - want.item()) < 1e-6


def test_shaped_mlp_sdf_level_set():
    """bench.shape_mlp_sdf: a random 8x256 softplus SkipConnMLP (the cfg2 / cfg4 SDF) becomes a
    rounded octahedron ~ (|x| + |y| + |z|) / sqrt(3) - const with its zero level set through
    (r, 0, 0), and stays 1-Lipschitz (sphere tracing never oversteps)."""
    import bench
    torch.manual_seed(0)
    m = R.SkipMLP(num_layers=8, hidden_size=256, out=1, freqs=16, activation="softplus")
    bench.shape_mlp_sdf(m, radius=0.3)
    with torch.no_grad():
        assert abs(m(torch.tensor([[0.3, 0.0, 0.0]]))[0, 0].item()) < 1e-2
        assert abs(m(torch.tensor([[0.0, -0.3, 0.0]]))[0, 0].item()) < 1e-2
        assert m(torch.zeros(1, 3))[0, 0].item() < -0.05
        # the diagonal point with the same L1 norm sits slightly inside: the softplus rounding
        # 2 log(1 + e^-|a x|) is largest on the coordinate planes
        t = 0.3 / 3
        assert -0.1 < m(torch.tensor([[t, t, t]]))[0, 0].item() < 0.0
        g = torch.Generator().manual_seed(0)
        p = torch.rand(512, 3, generator=g) * 2 - 1
        q = p + 1e-2 * F.normalize(torch.randn(512, 3, generator=g), dim=-1)
        lip = (m(q) - m(p)).abs().squeeze(-1) / (q - p).norm(dim=-1)
        assert lip.max().item() <= 1.0 + 1e-3, lip.max()


def test_sphere_ref_known_answers():
    """SphereRef (shapes/shapes.py:31-97): a ray from (0, 0, 2) down -z hits the unit sphere at
    t = 1, p = (0, 0, 1 + 1e-5), n = +z, wi = +z in the frame; a ray from inside takes the far
    root; a ray passing by misses (t from the unsquared discriminant: 6 here); t is in units of
    the unnormalised direction; intersect_limits gives both roots."""
    s = R.SphereRef()
    rays = torch.tensor([[0, 0, 2., 0, 0, -1], [0, 0, 2., 0, 1, 0], [0, 0, 0., 1, 0, 0],
                         [0, 3, 0, 0, -2, 0]])
    it, m = s.intersect(rays)
    assert m.tolist() == [True, False, True, True]
    assert torch.allclose(it.t, torch.tensor([1.0, 6.0, 1.0, 1.0]))  # |d| = 2 on the last
    assert torch.allclose(it.p[0], torch.tensor([0.0, 0.0, 1.0 + 1e-5]))
    assert torch.allclose(it.n[0], torch.tensor([0.0, 0.0, 1.0]))
    assert torch.allclose(it.wi[0], torch.tensor([0.0, 0.0, 1.0]), atol=1e-6)
    lo, hi, m2 = s.intersect_limits(rays)
    assert m2.tolist() == m.tolist()
    assert torch.allclose(lo[[0, 3]], torch.tensor([1.0, 1.0])) and torch.allclose(hi[[0, 3]], torch.tensor([3.0, 2.0]))
    assert math.isinf(hi[2].item())  # the root behind the origin
    assert s.intersect_test(rays).tolist() == m.tolist()


def test_renderer_point_light_ref_known_answer():
    """RendererPointLightRef (renderer/lighting.py:283-304): d = (loc - p) / (1e-7 + dist),
    Le = scale * ambient / (1e-7 + dist)^2."""
    light = R.RendererPointLightRef(location=[[0.0, 1.0, 4.0]], scale=100)
    it = R.Interaction(p=torch.tensor([[0.0, 0.0, 1.0]]))
    ds, le = light.sample_direction(it, torch.tensor([True]))
    dist = math.sqrt(10.0)
    assert torch.allclose(ds.d, torch.tensor([[0.0, 1.0, 3.0]]) / (1e-7 + dist))
    assert torch.allclose(le, torch.full((1, 3), 100 * 0.5 / (1e-7 + dist) ** 2))
    assert torch.allclose(ds.dist, torch.tensor([[dist]]))


def test_sphere_cloud_ref_one_sphere_is_the_sphere():
    """SphereCloudRef (shapes.py:99-206 statement by statement) with one sphere and t_max = inf
    equals SphereRef (shapes.py:31-97) on the hits -- the pin of the HIP SphereCloud's one-sphere
    case -- and misses keep t = inf."""
    import math
    g = torch.Generator().manual_seed(3)
    o = torch.tensor([0.0, 0.0, 2.0]) + 0.2 * torch.randn(1, 64, 1, 3, generator=g)
    d = torch.nn.functional.normalize(torch.cat([torch.rand(1, 64, 1, 2, generator=g) - 0.5,
                                                 -torch.ones(1, 64, 1, 1)], -1), dim=-1)
    rays = torch.cat([o, d], -1)
    cloud = R.SphereCloudRef(centers=[(0.1, 0.0, 0.0)], radii=0.5)
    sph = R.SphereRef((0.1, 0.0, 0.0), 0.5)
    ic, mc = cloud.intersect(rays)
    is_, ms = sph.intersect(rays)
    assert torch.equal(mc, ms) and 0 < int(mc.sum()) < 64
    assert torch.equal(ic.t[mc], is_.t[ms]) and torch.equal(ic.p[mc], is_.p[ms])
    assert torch.isinf(ic.t[~mc]).all()
    assert torch.equal(cloud.intersect_test(rays), sph.intersect_test(rays))
    assert math.isinf(float(ic.t[~mc][0])) if (~mc).any() else True
