"""PhysGaussian simulate + render driver -- drop-in for the reference's main.py.

    python main.py --config_path configs/lego.json [--n_grid 128] [--synthetic 100000]
                   [--output_path out/lego] [--white_background] [--save_pcd]

Same pipeline as main.py:164-335 of the reference: load Gaussians, sim-area
mask (inclusive bounds), world2grid, orbit camera (az 130, el 10, r 5.75, F16),
particle volumes, MPM_Simulator with the config's BCs plus the ground collider
at z = 0.4, then per frame ``steps_per_frame`` substeps, postprocess, render,
PNG.  Reference quirks are reproduced: render-space shift (F7), campos = the
world->camera translation (F8), black background unless --white_background
(F15).  Fixed here (they crash or write outside the run in the reference, F9):
a missing point_cloud2.ply is skipped and the debug PLY goes to output_path.
The per-frame state never leaves the GPU: grid2world runs fused in
gsmpm_mpm_world_outputs instead of the to_torch() D2H/H2D round trip.
"""
from __future__ import annotations

import json
import math
import os
import shutil
import sys
import time
from argparse import ArgumentParser

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from arguments import ModelParams, MPMParams, RenderParams  # noqa: E402
from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer  # noqa: E402
from gaussian_splatting.scene import GaussianModel  # noqa: E402
from gaussian_splatting.utils.graphics_utils import focal2fov, getProjectionMatrix, getWorld2View2  # noqa: E402
from gaussian_splatting.utils.system_utils import searchForMaxIteration  # noqa: E402
from internel_filling.filling import get_particle_volume  # noqa: E402
from mpm_solver.solver import MPM_Simulator  # noqa: E402
from utils.render_utils import TinyCam, to8b  # noqa: E402
from utils.transform_utils import (apply_cov_rotations, apply_inverse_cov_rotations, apply_inverse_rotations,  # noqa: E402
                                   apply_rotations, generate_rotation_matrices,
                                   get_camera_position_and_rotation,
                                   get_center_view_worldspace_and_observant_coordinate,
                                   particle_position_tensor_to_ply, undoshift2center111, undotransform2origin,
                                   world2grid)


def load_model(args):
    g = GaussianModel(sh_degree=3)
    if getattr(args, "synthetic", 0):
        print(f"Using {args.synthetic} synthetic Gaussians (seed 0)")
        return g.init_synthetic(args.synthetic, seed=0)
    it = args.loaded_iter if args.loaded_iter != -1 else searchForMaxIteration(
        os.path.join(args.model_path, "point_cloud"))
    print("Loading trained model at iteration {}".format(it))
    d = os.path.join(args.model_path, "point_cloud", "iteration_" + str(it))
    g.load_multiple_plys([os.path.join(d, "point_cloud.ply"), os.path.join(d, "point_cloud2.ply")])
    return g


def load_cameras(args):
    """main.py:50-82: cameras.json -> TinyCam list (only cameras[0] is used)."""
    path = os.path.join(args.model_path, "cameras.json")
    if not os.path.exists(path):
        # synthetic runs without a scene directory: lego camera 0 (800x800, fx = fy = 1111.11)
        infos = [{"width": 800, "height": 800, "fx": 1111.1110311937682, "fy": 1111.1110311937682,
                  "position": [0.0, 0.0, 4.0], "rotation": np.eye(3).tolist()}]
    else:
        with open(path) as f:
            infos = json.load(f)
    return [camera_from_info(ci) for ci in infos]


def camera_from_info(ci):
    """One cameras.json record -> TinyCam (main.py:58-80)."""
    w, h = ci["width"], ci["height"]
    fovx, fovy = focal2fov(ci["fx"], w), focal2fov(ci["fy"], h)
    center = np.array(ci["position"]).astype(np.float32)
    c2w = np.zeros((4, 4))
    c2w[:3, :3] = np.array(ci["rotation"])
    c2w[:3, 3] = center
    c2w[3, 3] = 1.0
    view = np.linalg.inv(c2w).transpose().astype(np.float32)
    proj = getProjectionMatrix(znear=0.01, zfar=100, fovX=fovx, fovY=fovy).numpy().transpose().astype(np.float32)
    return TinyCam(width=w, height=h, FovX=fovx, FovY=fovy, cam_center=center, view_mat=view,
                   full_proj_mat=view @ proj)


def modify_cam(cam: TinyCam, center_view_world_space, observant_coordinates, device="cuda"):
    """main.py:84-106: fixed orbit camera; campos = W2C translation T."""
    position, R = get_camera_position_and_rotation(130, 10, 5.75, center_view_world_space, observant_coordinates)
    tmp = np.zeros((4, 4))
    tmp[:3, :3] = R.tolist()
    tmp[:3, 3] = position.tolist()
    tmp[3, 3] = 1
    w2c = np.linalg.inv(tmp)
    Rv = w2c[:3, :3].transpose()
    T = w2c[:3, 3]
    proj = getProjectionMatrix(znear=0.01, zfar=100, fovX=cam.FovX, fovY=cam.FovY).transpose(0, 1).to(device)
    cam.view_mat = torch.tensor(getWorld2View2(Rv, T, np.array([0.0, 0.0, 0.0]), 1.0)).transpose(0, 1).to(device)
    cam.view_mat = cam.view_mat.to(torch.float32).contiguous()  # once here, not per render (the rasterizer needs it dense)
    cam.cam_center = T.astype(np.float32)
    cam.full_proj_mat = (cam.view_mat.unsqueeze(0).bmm(proj.unsqueeze(0))).squeeze(0).to(torch.float32)
    return cam


def render_frame(cam: TinyCam, pc: GaussianModel, mask, sim_means3D, sim_covs, bg_color, args, rotation_matrices,
                 pos_center, scaling_modifier=1.0, to_host=True):
    """main.py:108-157 (render-space transform with scaling_modifier = 1.0)."""
    settings = GaussianRasterizationSettings(
        image_height=cam.height, image_width=cam.width, tanfovx=math.tan(cam.FovX * 0.5),
        tanfovy=math.tan(cam.FovY * 0.5), bg=bg_color, scale_modifier=scaling_modifier, viewmatrix=cam.view_mat,
        projmatrix=cam.full_proj_mat, sh_degree=pc.active_sh_degree, campos=cam.cam_center, prefiltered=False,
        debug=args.debug)
    rasterizer = GaussianRasterizer(raster_settings=settings)
    means3D = apply_inverse_rotations(undotransform2origin(undoshift2center111(sim_means3D), scaling_modifier,
                                                           pos_center), rotation_matrices)
    covs = apply_inverse_cov_rotations(sim_covs / (scaling_modifier * scaling_modifier), rotation_matrices)
    image, _ = rasterizer(means3D=means3D, means2D=None, shs=pc.get_features[mask], colors_precomp=None,
                          opacities=pc.get_opacity[mask], scales=None, rotations=None, cov3D_precomp=covs)
    return image.detach().cpu().numpy().transpose(1, 2, 0) if to_host else image


def save_frame(frame, save_path, fid, save_seq):
    from PIL import Image
    save_seq.append(frame)
    Image.fromarray(to8b(frame)).save(os.path.join(save_path, f"{fid:04d}.png"))


class FrameWriter:
    """main.py:157-161 without the stalls: each rendered image is copied into a
    pinned host buffer on the render's stream (non-blocking) and encoded to PNG
    on a worker thread once its copy event completes, while the GPU already
    simulates the next frame.  Same files, same frame order."""

    def __init__(self, save_path, save_seq, workers=4):
        from concurrent.futures import ThreadPoolExecutor
        self.path, self.seq = save_path, save_seq
        self.pool = ThreadPoolExecutor(max_workers=workers)
        self.jobs = []

    def submit(self, image, fid):
        host = torch.empty(image.shape, dtype=image.dtype, pin_memory=True)
        host.copy_(image, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        slot = len(self.seq)
        self.seq.append(None)

        def work():
            ev.synchronize()
            frame = host.numpy().transpose(1, 2, 0)
            self.seq[slot] = frame
            from PIL import Image
            Image.fromarray(to8b(frame)).save(os.path.join(self.path, f"{fid:04d}.png"))

        self.jobs.append(self.pool.submit(work))

    def close(self):
        for j in self.jobs:
            j.result()
        self.pool.shutdown()


def simulate(model_args, sim_args, render_args):
    dev = torch.device("cuda")
    gaussians = load_model(model_args)
    cams = load_cameras(model_args)
    rot = generate_rotation_matrices([torch.tensor(0.0)], [torch.tensor(0.0)], device=dev)
    rotated = apply_rotations(gaussians.get_xyz, rot)
    bound = torch.tensor(np.array(sim_args.sim_area)).to(dev)
    mask = torch.logical_and((rotated <= bound[1]).all(dim=1), (rotated >= bound[0]).all(dim=1))
    print(f"Number of simulatable Gaussians: {int(mask.sum())}")
    background = torch.tensor([1, 1, 1] if render_args.white_background else [0, 0, 0], dtype=torch.float32,
                              device=dev)
    out_images = os.path.join(render_args.output_path, "images")
    os.makedirs(out_images, exist_ok=True)
    seq = []
    particle_position_tensor_to_ply(rotated, os.path.join(render_args.output_path, "rotated_particles.ply"))

    sim_means3D = rotated[mask].detach()
    sim_covs = apply_cov_rotations(gaussians.get_covariance()[mask].detach(), rot)
    xg, pos_center, s = world2grid(sim_means3D, sim_args)
    covs_g = sim_covs * (s * s)
    center_w, obs = get_center_view_worldspace_and_observant_coordinate(
        torch.tensor([0.5, 0.5, 0.5]).reshape((1, 3)).to(dev), torch.tensor([0, 0, 1]).reshape((1, 3)).to(dev), rot, s,
        pos_center)
    cam = modify_cam(cams[0], center_w, obs, device=dev)
    cam.toCuda(dev)
    vols = get_particle_volume(xg, sim_args)
    solver = MPM_Simulator(xg, covs_g, vols, sim_args)
    solver.set_boundary_conditions(sim_args.boundary_conditions, sim_args)
    solver.add_surface_collider((0.0, 0.0, 0.4), (0.0, 0.0, 1.0))

    writer = FrameWriter(out_images, seq)
    writer.submit(render_frame(cam, gaussians, mask, sim_means3D, sim_covs, background, model_args, rot, pos_center,
                               to_host=False), 0)
    t0 = time.time()
    for fid in range(1, render_args.num_frames + 1):
        for _ in range(sim_args.steps_per_frame):
            solver.p2g2p(sim_args.substep_dt)
        solver.postprocess()
        sim_means3D, sim_covs = solver._sim.world_outputs(s, pos_center.tolist(), render_space=False)
        if render_args.save_pcd and fid % render_args.save_pcd_interval == 0:
            g2 = GaussianModel(3, device=dev)
            g2._set(*[t.detach().cpu().numpy() for t in (gaussians._xyz, gaussians._features_dc,
                                                          gaussians._features_rest, gaussians._opacity,
                                                          gaussians._scaling, gaussians._rotation)])
            g2._xyz[mask] = sim_means3D
            g2.save_ply(os.path.join(render_args.output_path, "point_cloud", f"iteration_{fid}", "point_cloud.ply"))
        writer.submit(render_frame(cam, gaussians, mask, sim_means3D, sim_covs, background, model_args, rot,
                                   pos_center, to_host=False), fid)
        if fid % 10 == 0 or fid == render_args.num_frames:
            el = time.time() - t0
            print(f"frame {fid}/{render_args.num_frames}  {fid / el:.1f} fps (sim+render+png)", flush=True)
    writer.close()
    print(f"{render_args.num_frames / (time.time() - t0):.1f} fps with every PNG written", flush=True)
    if render_args.save_pcd:
        for name in ("cameras.json", "cfg_args", "input.ply"):
            src = os.path.join(model_args.model_path, name)
            if os.path.exists(src):
                shutil.copy(src, os.path.join(render_args.output_path, name))
    if shutil.which("ffmpeg"):
        os.system(f"ffmpeg -framerate 25 -i {out_images}/%04d.png -c:v libx264 -vf \"pad=ceil(iw/2)*2:ceil(ih/2)*2\" "
                  f"-y -pix_fmt yuv420p {render_args.output_path}/simulated.mp4")
    print("Done.")


def main(argv=None):
    cp = ArgumentParser(add_help=False)
    cp.add_argument("--config_path", type=str, required=True)
    cargs, rest = cp.parse_known_args(argv)
    with open(cargs.config_path) as f:
        config = json.load(f)
    parser = ArgumentParser(description="Simulation parameters")
    m = ModelParams(parser, config["model"])
    s = MPMParams(parser, config["mpm"])
    r = RenderParams(parser, config["render"])
    args = parser.parse_args(rest)
    simulate(m.extract(args), s.extract(args), r.extract(args))


if __name__ == "__main__":
    main()
