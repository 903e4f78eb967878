"""extra.py drop-in: physical-parameter identification (SystemIndentifier,
reference extra.py:69-348) on libgsmpm.so -- the differentiable MPM
(MPM_Simulator(fitting=True) -> gsmpm_fit_*) and the rasterizer forward +
backward (GaussianRasterizer -> gsmpm_raster_forward / _backward).

Same structure, loop and numerics as the reference:
  per iteration: world2grid (+-0.3 padding), particle volumes, a fresh
  MPM_Simulator(fitting=True) + set_bc_ground_only; frame 0 fits the
  Gaussians' appearance (Adam); frames 1..19 run 30 forward substeps of
  0.03/30, render level 30, loss = 0.8 L1 + 0.2 SSIM, torch backward through
  the rasterizer, set_grads, 30 backward substeps, learn (clipped SGD on logE
  and y), cycle_init; E and nu are read back after every frame.
Differences, each deliberate:
  * extra.py:207 calls p2g2p(dt, s), which the reference's p2g2p does not
    accept; the drop-in routes it to p2g2p_forward(dt, s).
  * the reference's data (data_extra/, models_extra/torus) is not in the
    repository: --synthetic N builds an N-Gaussian torus, a ring of cameras
    and ground-truth frames rendered from the same simulator at --E_true.
    The on-disk loaders (camera.json, frame.json, physical.json, PNGs,
    static_gaussians/point_cloud.ply, init_velocity.json) are kept for real data.
"""
from __future__ import annotations

import json
import math
import os
import random
import sys
import time
from argparse import ArgumentParser
from copy import deepcopy

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from arguments import MPMParams  # noqa: E402
from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer  # noqa: E402
from gaussian_splatting.scene import GaussianModel  # noqa: E402
from gaussian_splatting.scene.cameras import Camera  # noqa: E402
from gaussian_splatting.scene.dataset_readers import CameraInfo, getNerfppNorm  # noqa: E402
from gaussian_splatting.utils.graphics_utils import focal2fov  # noqa: E402
from gaussian_splatting.utils.loss_utils import l1_loss, ssim  # noqa: E402
from internel_filling.filling import get_particle_volume  # noqa: E402
from mpm_solver.solver import MPM_Simulator  # noqa: E402

data_root = "data_extra/mpm_synthetic"
model_root = "models_extra"

image_width = 512
image_height = 512
image_bg = np.array([1, 1, 1])

grid_extent = 2.0
n_grid = 50

G = np.array([0.0, -9.81, 0.0])

train_num_frames = 20
test_num_frames = 10

total_iters = 300


def _bg_cuda():
    return torch.tensor(image_bg, dtype=torch.float32, device="cuda")


class SystemIndentifier:
    def __init__(self, data_path, model_path, sim_args, args, synthetic=None):
        self.sim_args = sim_args
        self.args = args
        self.total_iters = getattr(args, "iters", total_iters)
        self.image_bg_cuda = _bg_cuda()
        if synthetic is not None:
            self.synthesize(**synthetic)
        else:
            self.load_data_and_cameras(data_path)
            self.load_physics_info(data_path)
            self.load_model(model_path)

    # ------------------------------------------------------------ real data --
    def load_data_and_cameras(self, data_path):
        """extra.py:83-154: per-frame cameras + RGBA images composited on the background."""
        from PIL import Image
        from gaussian_splatting.utils.general_utils import PILtoTorch
        with open(os.path.join(data_path, "camera.json"), "r") as cam_file:
            cameras = json.load(cam_file)
        cam_infos_all = []
        for frame_id in range(train_num_frames + test_num_frames):
            cam_infos = []
            for cam_id, camera in enumerate(cameras):
                intrinsic = np.array(camera["K"])
                c2w = deepcopy(np.array(camera["c2w"]))
                c2w[:3, 1:3] *= -1
                w2c = np.linalg.inv(c2w)
                R = np.transpose(w2c[:3, :3])
                T = w2c[:3, 3]
                FovX = focal2fov(intrinsic[0][0], image_width)
                FovY = focal2fov(intrinsic[1][1], image_height)
                cam_name = camera["camera"]
                image_path = os.path.join(data_path, cam_name, f"{frame_id:03}.png")
                im_data = np.array(Image.open(image_path).convert("RGBA"))
                norm_data = im_data / 255.0
                arr = norm_data[:, :, :3] * norm_data[:, :, 3:4] + image_bg * (1 - norm_data[:, :, 3:4])
                image = Image.fromarray(np.array(arr * 255.0, dtype=np.byte), "RGB")
                cam_infos.append(CameraInfo(uid=cam_id, R=R, T=T, FovY=FovY, FovX=FovX, image=image,
                                            image_path=image_path, image_name=f"{cam_name}_{frame_id:03}.png",
                                            width=image_width, height=image_height))
            cam_infos_all.append(cam_infos)
        self.spatial_lr_scale = getNerfppNorm(cam_infos_all[0])["radius"]
        self.cameras_all = []
        for frame_id in range(train_num_frames + test_num_frames):
            camera_list = []
            for cid, c in enumerate(cam_infos_all[frame_id]):
                gt_image = PILtoTorch(c.image, (image_width, image_height))[:3, ...]
                camera_list.append(Camera(colmap_id=c.uid, R=c.R, T=c.T, FoVx=c.FovX, FoVy=c.FovY, image=gt_image,
                                          gt_alpha_mask=None, image_name=c.image_name, uid=cid, data_device="cuda"))
            self.cameras_all.append(camera_list)
        self.dt = []
        with open(os.path.join(data_path, "frame.json"), "r") as file:
            frame_time_steps = json.load(file)
            for fid in range(1, len(frame_time_steps)):
                self.dt.append(frame_time_steps[fid][f"{fid:03d}"] - frame_time_steps[fid - 1][f"{fid - 1:03d}"])

    def load_physics_info(self, data_path):
        with open(os.path.join(data_path, "physical.json"), "r") as physical_file:
            self.physics_info = json.load(physical_file)

    def load_model(self, model_path):
        self.gaussians = GaussianModel(sh_degree=3)
        self.gaussians.load_ply(os.path.join(model_path, "static_gaussians", "point_cloud.ply"))
        self.n_particles = self.gaussians.get_xyz.shape[0]
        with open(os.path.join(model_path, "init_velocity.json"), "r") as file:
            self.init_v = torch.tensor(json.load(file)).repeat(self.n_particles, 1)

    # ------------------------------------------------------- synthetic data --
    def synthesize(self, n, E_true, nu_true=None, n_cams=4, size=256, seed=0, v0=(0.0, -1.0, 0.0)):
        """an n-Gaussian torus (R = 0.3, r = 0.1), a ring of
        n_cams cameras, and ground-truth frames rendered from this simulator at
        E_true (frames 1.. by the same 30-substep forward + cycle_init the loop uses)."""
        global image_width, image_height
        image_width = image_height = size
        rng = np.random.default_rng(seed)
        th, ph = rng.uniform(0, 2 * np.pi, n), rng.uniform(0, 2 * np.pi, n)
        r = 0.1 * np.sqrt(rng.uniform(0, 1, n))
        xyz = np.stack([(0.3 + r * np.cos(ph)) * np.cos(th), r * np.sin(ph), (0.3 + r * np.cos(ph)) * np.sin(th)], 1)
        g = GaussianModel(3)
        k = 15
        rot = rng.normal(0, 1, (n, 4))
        dc = np.stack([0.8 + 0.6 * np.cos(th), 0.2 + 0.6 * np.sin(ph), 0.9 - 0.5 * np.cos(2 * th)], 1)[:, None, :]
        g._set(xyz, dc, rng.normal(0, 0.02, (n, k, 3)), np.full((n, 1), 3.0), np.full((n, 3), -4.0),
               rot / np.linalg.norm(rot, axis=1, keepdims=True))
        self.gaussians = g
        self.n_particles = n
        self.init_v = torch.tensor(list(v0)).repeat(n, 1)
        fov = 2 * math.atan(0.45)
        cams = []
        for c in range(n_cams):
            az = 2 * math.pi * c / n_cams
            pos = np.array([2.2 * math.cos(az), 1.0, 2.2 * math.sin(az)])
            f = -pos / np.linalg.norm(pos)
            rr = np.cross(f, [0.0, 1.0, 0.0])
            rr /= np.linalg.norm(rr)
            d = np.cross(f, rr)
            c2w = np.eye(4)
            c2w[:3, 0], c2w[:3, 1], c2w[:3, 2], c2w[:3, 3] = rr, d, f, pos
            w2c = np.linalg.inv(c2w)
            cams.append((np.transpose(w2c[:3, :3]), w2c[:3, 3]))
        self.spatial_lr_scale = 2.2 * 1.1
        blank = torch.zeros(3, size, size)
        mk = lambda R, T, img, name, cid: Camera(colmap_id=cid, R=R, T=T, FoVx=fov, FoVy=fov, image=img,
                                                 gt_alpha_mask=None, image_name=name, uid=cid, data_device="cuda")
        base = [mk(R, T, blank, f"cam{c}", c) for c, (R, T) in enumerate(cams)]
        # ground truth: the same pipeline at E_true
        sa = deepcopy(self.sim_args)
        sa.E = E_true
        sa.nu = nu_true if nu_true is not None else self.sim_args.nu
        with torch.no_grad():
            sim_means3D = self.gaussians.get_xyz
            sim_covs = self.gaussians.get_covariance()
            tm = self.world2grid(sim_means3D)
            vol = get_particle_volume(tm.detach(), sa)
            sim = MPM_Simulator(tm, sim_covs * (self.scaling_modifier ** 2), vol, sa, init_v=self.init_v.cuda())
            sim.set_bc_ground_only()
            self.cameras_all = []
            for fid in range(train_num_frames + test_num_frames):
                if fid == 0:
                    means, covs = sim_means3D, sim_covs
                else:
                    for s in range(30):
                        sim.p2g2p_forward(0.03 / 30, s)
                    sim.postprocess_forward()
                    means, covs = self.grid2world(sim.mpm_state.particle_xyz.to_torch()[30],
                                                  sim.mpm_state.particle_cov.to_torch(), sa)
                    sim.mpm_state.cycle_init()
                frame = []
                for cam in base:
                    img = self.render(cam, self.gaussians, means, covs)
                    frame.append(mk(cam.R, cam.T, img.detach().cpu(), f"{cam.image_name}_{fid:03d}", cam.uid))
                self.cameras_all.append(frame)
        self.E_true, self.nu_true = E_true, sa.nu

    # ------------------------------------------------------------- training --
    def train(self, log=print):
        self.training_setup()
        optimized_E, optimized_nu = None, None
        history = []
        for iteration in range(1, self.total_iters + 1):
            sim_means3D = self.gaussians.get_xyz
            sim_covs = self.gaussians.get_covariance()
            init_velocities = self.init_v.float().cuda()
            transformed_sim_means3D = self.world2grid(sim_means3D)
            transformed_sim_covs = sim_covs * (self.scaling_modifier * self.scaling_modifier)
            sim_volumes = get_particle_volume(transformed_sim_means3D.detach(), self.sim_args)
            self.sim_args.E = optimized_E if optimized_E is not None else self.sim_args.E
            self.sim_args.nu = optimized_nu if optimized_E is not None else self.sim_args.nu
            mpm_solver = MPM_Simulator(transformed_sim_means3D.detach(), transformed_sim_covs.detach(), sim_volumes,
                                       self.sim_args, init_v=init_velocities)
            mpm_solver.set_bc_ground_only()
            for fid in range(train_num_frames):
                cam_id = random.randint(1, len(self.cameras_all[fid])) - 1
                viewpoint_cam = self.cameras_all[fid][cam_id]
                gt_image = viewpoint_cam.original_image
                if fid == 0:  # optimize the Gaussians' appearance
                    rendered_image = self.render(viewpoint_cam, self.gaussians, sim_means3D, sim_covs)
                    loss = 0.8 * l1_loss(rendered_image, gt_image) + 0.2 * ssim(rendered_image, gt_image)
                    loss.backward()
                    self.gaussians.optimizer.step()
                    self.gaussians.optimizer.zero_grad(set_to_none=True)
                else:  # optimize the physical parameters
                    for s in range(30):
                        mpm_solver.p2g2p(0.03 / 30, s)  # extra.py:207 (SURVEY F9 routed to p2g2p_forward)
                    mpm_solver.postprocess_forward()
                    mpm_sim_means3D = mpm_solver.mpm_state.particle_xyz.to_torch()[30].cuda().requires_grad_(True)
                    mpm_sim_covs = mpm_solver.mpm_state.particle_cov.to_torch().cuda().requires_grad_(True)
                    sim_means3D, sim_covs = self.grid2world(mpm_sim_means3D, mpm_sim_covs, self.sim_args)
                    rendered_image = self.render(viewpoint_cam, self.gaussians, sim_means3D, sim_covs)
                    loss = 0.8 * l1_loss(rendered_image, gt_image) + 0.2 * ssim(rendered_image, gt_image)
                    loss.backward()
                    mpm_solver.clear_grads()
                    mpm_solver.mpm_state.set_grads(mpm_sim_means3D.grad.cpu().numpy().astype(np.float32),
                                                   mpm_sim_covs.grad.cpu().numpy().astype(np.float32))
                    mpm_solver.postprocess_backward()
                    for s in reversed(range(30)):
                        mpm_solver.p2g2p_backward(0.03 / 30, s)
                    mpm_solver.learn()
                    mpm_solver.mpm_state.cycle_init()
                optimized_E = 10 ** mpm_solver.mpm_model.logE.to_torch().mean().item()
                optimized_nu = 0.49 / (1.0 + torch.exp(-mpm_solver.mpm_model.y.to_torch().mean())).item()
                history.append((iteration, fid, float(loss.item()), optimized_E, optimized_nu))
                log(f"iter {iteration} frame {fid}: loss {loss.item():.5f} E {optimized_E:.6g} nu {optimized_nu:.4f}")
        return history

    def render(self, viewpoint_camera, pc, sim_means3D, sim_covs):
        """extra.py:260-305."""
        screenspace_points = torch.zeros_like(pc.get_xyz, dtype=pc.get_xyz.dtype, requires_grad=True,
                                              device="cuda") + 0
        try:
            screenspace_points.retain_grad()
        except Exception:
            pass
        tanfovx = math.tan(viewpoint_camera.FoVx * 0.5)
        tanfovy = math.tan(viewpoint_camera.FoVy * 0.5)
        raster_settings = GaussianRasterizationSettings(
            image_height=int(viewpoint_camera.image_height), image_width=int(viewpoint_camera.image_width),
            tanfovx=tanfovx, tanfovy=tanfovy, bg=self.image_bg_cuda, scale_modifier=1.0,
            viewmatrix=viewpoint_camera.world_view_transform, projmatrix=viewpoint_camera.full_proj_transform,
            sh_degree=pc.active_sh_degree, campos=viewpoint_camera.camera_center, prefiltered=False, debug=False)
        rasterizer = GaussianRasterizer(raster_settings=raster_settings)
        rendered_image, _ = rasterizer(means3D=sim_means3D, means2D=screenspace_points, shs=pc.get_features,
                                       colors_precomp=None, opacities=pc.get_opacity, scales=None, rotations=None,
                                       cov3D_precomp=sim_covs)
        return rendered_image

    def training_setup(self):
        """extra.py:308-316 (Adam over the Gaussians' parameters)."""
        g = self.gaussians
        for t in (g._xyz, g._features_dc, g._features_rest, g._opacity, g._scaling):
            t.requires_grad_(True)
        lr = [{"params": [g._xyz], "lr": 0.0000016 * self.spatial_lr_scale, "name": "xyz"},
              {"params": [g._features_dc], "lr": 0.0025, "name": "f_dc"},
              {"params": [g._features_rest], "lr": 0.0025 / 20.0, "name": "f_rest"},
              {"params": [g._opacity], "lr": 0.05, "name": "opacity"},
              {"params": [g._scaling], "lr": 0.005, "name": "scaling"}]
        g.optimizer = torch.optim.Adam(lr, lr=0.0, eps=1e-15)

    def world2grid(self, means3D):
        """extra.py:319-325."""
        pos_min, pos_max = means3D.min(dim=0)[0] - 0.3, means3D.max(dim=0)[0] + 0.3
        self.pos_center = ((pos_min + pos_max) / 2.0).detach()
        self.scaling_modifier = grid_extent / 2.0 / (pos_max - pos_min).max().detach()
        return (means3D - self.pos_center) * self.scaling_modifier + torch.ones(3).cuda() * grid_extent / 2.0

    def grid2world(self, means3D, covs, sim_args):
        """extra.py:328-331."""
        transformed_means3D = (means3D - torch.ones(3).cuda() * sim_args.grid_extent / 2.0) / self.scaling_modifier \
            + self.pos_center
        transformed_covs = covs / (self.scaling_modifier * self.scaling_modifier)
        return transformed_means3D, transformed_covs.view(-1, 6)


if __name__ == "__main__":
    parser = ArgumentParser(add_help=False)
    parser.add_argument("--scene", type=str, default="torus")
    parser.add_argument("--output_path", type=str, default="outputs_extra/torus_debug")
    parser.add_argument("--synthetic", type=int, default=0, help="N torus Gaussians instead of data_extra/")
    parser.add_argument("--E_true", type=float, default=1e5)
    parser.add_argument("--image_size", type=int, default=256)
    parser.add_argument("--iters", type=int, default=total_iters)
    sim_args = MPMParams(parser)
    args = parser.parse_args()
    for k in ("E", "nu", "density", "n_grid", "grid_extent"):  # CLI overrides of the MPMParams group
        setattr(sim_args, k, getattr(args, k))
    sim_args.fitting = True
    os.makedirs(args.output_path, exist_ok=True)
    syn = dict(n=args.synthetic, E_true=args.E_true, size=args.image_size) if args.synthetic else None
    si = SystemIndentifier(os.path.join(data_root, args.scene), os.path.join(model_root, args.scene), sim_args, args,
                           synthetic=syn)
    t0 = time.perf_counter()
    hist = si.train()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    with open(os.path.join(args.output_path, "history.json"), "w") as f:
        json.dump({"history": hist, "seconds": el, "E_true": getattr(si, "E_true", None)}, f)
    print(f"{len(hist)} frames in {el:.2f} s; final E {hist[-1][3]:.6g}")
