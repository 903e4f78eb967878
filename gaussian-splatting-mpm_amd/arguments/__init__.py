"""JSON-seeded argparse groups (arguments/__init__.py:1-100 of the reference).

Semantics kept for the drop-in CLI: every attribute of a group becomes a
``--flag`` typed by its default; JSON values replace defaults; CLI overrides
JSON; JSON keys a group does not declare are ignored (which is why lego.json's
``model.white_background`` never reaches RenderParams).  A leading
underscore adds a one-letter short flag.  Additions (all default-off):
MPMParams.jelly_fcr (fix SURVEY F3), ModelParams.synthetic (generate
Gaussians when the scene's PLY is absent / an LFS pointer).
"""
from argparse import ArgumentParser


class GroupParams:
    pass


class ParamGroup:
    def __init__(self, parser: ArgumentParser, name: str, json_params=None):
        grp = parser.add_argument_group(name)
        json_params = json_params or {}
        for attr, default in vars(self).items():
            short = attr.startswith("_")
            key = attr[1:] if short else attr
            kind = type(default)
            value = json_params.get(key, default)
            names = ["--" + key] + (["-" + key[0:1]] if short else [])
            if kind == bool:
                grp.add_argument(*names, default=value, action="store_true")
            else:
                grp.add_argument(*names, default=value, type=kind)

    def extract(self, args):
        out = GroupParams()
        mine = vars(self)
        for k, v in vars(args).items():
            if k in mine or ("_" + k) in mine:
                setattr(out, k, v)
        return out


class ModelParams(ParamGroup):
    def __init__(self, parser, json_params=None):
        self.model_path = ""
        self.loaded_iter = -1
        self.debug = False
        self.synthetic = 0  # >0: N synthetic lego-like Gaussians instead of the PLY
        super().__init__(parser, "Loading Parameters", json_params)


class MPMParams(ParamGroup):
    def __init__(self, parser, json_params=None):
        self.view_area = []
        self.sim_area = [[-1.0, -1.0, -1.0], [1.0, 1.0, 1.0]]
        self.mask = []
        self.E = 2e6
        self.nu = 0.4
        self.viscosity = 0.05
        self.material = "jelly"
        self.gravity = [0.0, -9.81, 0.0]
        self.density = 1000.0
        self.n_grid = 50
        self.grid_extent = 2.0
        self.substep_dt = 0.0006
        self.frame_dt = 0.03
        self.rotation_degree = [0.0, 0.0, 0.0]
        self.boundary_conditions = []
        self.fitting = False
        self.jelly_fcr = False
        super().__init__(parser, "MPM Parameters", json_params)

    def extract(self, args):
        g = super().extract(args)
        g.steps_per_frame = int(g.frame_dt / g.substep_dt)  # arguments/__init__.py:83
        return g


class RenderParams(ParamGroup):
    def __init__(self, parser, json_params=None):
        self.output_path = ""
        self.white_background = False
        self.view_cam_idx = 10
        self.num_frames = 60
        self.save_pcd = False
        self.save_pcd_interval = 10
        super().__init__(parser, "Render Parameters", json_params)
