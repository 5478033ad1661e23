"""Parameter classes and a libconfig-subset reader for the driver_mgmc configuration files.

Mirrors auxilliary/parameters.{hh,cc} of the reference (GeneralParameters, LatticeParameters,
MultigridParameters, SamplingParameters, PriorParameters, ConstantCorrelationLengthModelParameters,
MeasurementParameters; parameters.cc:21-337).  libconfig++ is not available in this image, so the
subset of the libconfig grammar used by parameters_template.cfg / measurements_template.cfg
(groups, scalars, strings, booleans, arrays, // and /* */ comments) is parsed here.
"""
from __future__ import annotations

import math
import re
from dataclasses import dataclass, field
from typing import Any

_TOKEN = re.compile(r"""
    (?P<ws>\s+) |
    (?P<comment>//[^\n]*|\#[^\n]*|/\*.*?\*/) |
    (?P<string>"(?:[^"\\]|\\.)*") |
    (?P<number>[-+]?(?:\d+\.\d*|\.\d+|\d+)(?:[eE][-+]?\d+)?[Ll]?) |
    (?P<name>[A-Za-z_][A-Za-z0-9_\-]*) |
    (?P<punct>[={}\[\]();,:])
""", re.VERBOSE | re.DOTALL)


class ConfigError(ValueError):
    pass


class MeasurementFileError(ConfigError):
    """The measurements file named by measurements.filename cannot be opened (parameters.cc:273-276)."""


def _tokenize(text: str):
    pos = 0
    out = []
    while pos < len(text):
        m = _TOKEN.match(text, pos)
        if not m:
            raise ConfigError(f"unexpected character {text[pos]!r} at offset {pos}")
        pos = m.end()
        kind = m.lastgroup
        if kind in ("ws", "comment"):
            continue
        out.append((kind, m.group(kind)))
    return out


class _Parser:
    def __init__(self, tokens):
        self.t = tokens
        self.i = 0

    def peek(self):
        return self.t[self.i] if self.i < len(self.t) else (None, None)

    def take(self, value=None):
        tok = self.peek()
        if tok[0] is None or (value is not None and tok[1] != value):
            raise ConfigError(f"expected {value!r}, got {tok[1]!r}")
        self.i += 1
        return tok

    def settings(self, closing=None) -> dict:
        out = {}
        while True:
            kind, val = self.peek()
            if kind is None or val == closing:
                return out
            name = self.take()[1]
            sep = self.take()[1]
            if sep not in ("=", ":"):
                raise ConfigError(f"expected '=' after {name}")
            out[name] = self.value()
            if self.peek()[1] in (";", ","):
                self.i += 1

    def value(self) -> Any:
        kind, val = self.peek()
        if val == "{":
            self.take("{")
            v = self.settings("}")
            self.take("}")
            return v
        if val in ("[", "("):
            close = "]" if val == "[" else ")"
            self.take(val)
            items = []
            while self.peek()[1] != close:
                items.append(self.value())
                if self.peek()[1] == ",":
                    self.i += 1
            self.take(close)
            return items
        self.i += 1
        if kind == "string":
            return bytes(val[1:-1], "utf-8").decode("unicode_escape")
        if kind == "number":
            v = val.rstrip("Ll")
            if re.fullmatch(r"[-+]?\d+", v):
                return int(v)
            return float(v)
        if kind == "name":
            low = val.lower()
            if low in ("true", "false"):
                return low == "true"
        raise ConfigError(f"unexpected token {val!r}")


def parse_config(text: str) -> dict:
    """Parse libconfig text into nested dicts / lists / scalars."""
    return _Parser(_tokenize(text)).settings()


def read_config(filename: str) -> dict:
    with open(filename) as fh:
        return parse_config(fh.read())


def _get(cfg: dict, path: str):
    node = cfg
    for key in path.split("."):
        if not isinstance(node, dict) or key not in node:
            raise ConfigError(f"setting '{path}' not found")
        node = node[key]
    return node


@dataclass
class GeneralParameters:
    dim: int = 2
    do_cholesky: bool = False
    do_ssor: bool = False
    do_multigridmc: bool = True
    save_posterior_statistics: bool = False
    measure_convergence: bool = False
    operator_name: str = "prior"

    @classmethod
    def from_config(cls, cfg: dict) -> "GeneralParameters":
        g = _get(cfg, "general")
        return cls(int(g["dim"]), bool(g["do_cholesky"]), bool(g["do_ssor"]), bool(g["do_multigridmc"]),
                   bool(g["save_posterior_statistics"]), bool(g.get("measure_convergence", False)),
                   str(g["operator"]))


@dataclass
class LatticeParameters:
    nx: int = 32
    ny: int = 32
    nz: int = 32

    @classmethod
    def from_config(cls, cfg: dict) -> "LatticeParameters":
        g = _get(cfg, "lattice")
        return cls(int(g["nx"]), int(g["ny"]), int(g.get("nz", 0)))


@dataclass
class MultigridParameters:
    """parameters.hh:145-174 (MultigridParameters)."""
    nlevel: int = 4
    smoother: str = "SOR"
    coarse_solver: str = "SSOR"
    npresmooth: int = 1
    npostsmooth: int = 1
    ncoarsesmooth: int = 1
    omega: float = 1.0
    cycle: int = 1
    coarse_scaling: float = 1.0
    verbose: int = 0

    @classmethod
    def from_config(cls, cfg: dict) -> "MultigridParameters":
        g = _get(cfg, "multigrid")
        return cls(int(g["nlevel"]), str(g["smoother"]), str(g["coarse_solver"]), int(g["npresmooth"]),
                   int(g["npostsmooth"]), int(g["ncoarsesmooth"]), float(g["omega"]), int(g["cycle"]),
                   float(g["coarse_scaling"]), int(g.get("verbose", 0)))


@dataclass
class SamplingParameters:
    nsamples: int = 100
    nwarmup: int = 10
    nstepsconvergence: int = 16
    nsamplesconvergence: int = 100

    @classmethod
    def from_config(cls, cfg: dict) -> "SamplingParameters":
        g = _get(cfg, "sampling")
        return cls(int(g["timeseries"]["nsamples"]), int(g["timeseries"]["nwarmup"]),
                   int(g["convergence"]["nsteps"]), int(g["convergence"]["nsamples"]))


@dataclass
class PriorParameters:
    pde_model: str = "shiftedlaplace_fd"
    correlationlength_model: str = "constant"

    @classmethod
    def from_config(cls, cfg: dict) -> "PriorParameters":
        g = _get(cfg, "prior")
        return cls(str(g["pdemodel"]), str(g["correlationlengthmodel"]))


@dataclass
class ConstantCorrelationLengthModelParameters:
    Lambda: float = 0.2

    @property
    def kappa_sq(self) -> float:
        # correlationlength_model.hh:52
        return 1.0 / math.pow(self.Lambda, 2)

    @classmethod
    def from_config(cls, cfg: dict) -> "ConstantCorrelationLengthModelParameters":
        return cls(float(_get(cfg, "constantcorrelationlengthmodel")["Lambda"]))


@dataclass
class PeriodicCorrelationLengthModelParameters:
    """parameters.cc:224-243 (Lambda_max >= Lambda_min > 0, else the reference exits with -1)."""
    Lambda_min: float = 0.2
    Lambda_max: float = 0.4

    @classmethod
    def from_config(cls, cfg: dict) -> "PeriodicCorrelationLengthModelParameters":
        g = _get(cfg, "periodiccorrelationlengthmodel")
        out = cls(float(g["Lambda_min"]), float(g["Lambda_max"]))
        if not out.Lambda_max >= out.Lambda_min:
            raise ConfigError("ERROR: upper bound on correlation length has to exceed lower bound.")
        if not out.Lambda_min > 0:
            raise ConfigError("ERROR: lower bound on correlation length has to be positive.")
        return out


@dataclass
class MeasurementParameters:
    radius: float = 0.0
    sample_location: list = field(default_factory=lambda: [0.5, 0.5])
    variance_scaling: float = 1.0
    measure_global: bool = False
    mean_global: float = 1.0
    variance_global: float = 0.01
    filename: str = ""
    dim: int = 2
    n: int = 0
    measurement_locations: list = field(default_factory=list)
    mean: list = field(default_factory=list)
    variance: list = field(default_factory=list)

    @classmethod
    def from_config(cls, cfg: dict, base_dir: str | None = None) -> "MeasurementParameters":
        """parameters.cc:245-300.  The measurements file is opened as given, i.e. relative to the
        working directory, like the reference's readFile(filename); only if that fails is it looked
        up next to the configuration file (base_dir).  A file found in neither place raises
        MeasurementFileError with the reference's message (parameters.cc:273-276 prints it and
        exits with -1): a posterior without its measurements is never built silently."""
        import os
        g = _get(cfg, "measurements")
        p = cls(float(g["radius"]), [float(v) for v in g["sample_location"]], float(g["variance_scaling"]),
                bool(g["measure_global"]), float(g["mean_global"]), float(g["variance_global"]),
                str(g["filename"]))
        candidates = [p.filename]
        if base_dir is not None and not os.path.isabs(p.filename):
            candidates.append(os.path.join(base_dir, p.filename))
        path = next((c for c in candidates if os.path.isfile(c)), None)
        if path is None:
            raise MeasurementFileError(f"ERROR opening configuration file with measurements: '{p.filename}'.")
        m = read_config(path)
        p.dim = int(m["dim"])
        p.n = int(m["n"])
        loc = [float(v) for v in m["measurement_locations"]]
        p.measurement_locations = [loc[p.dim * k:p.dim * (k + 1)] for k in range(p.n)]
        p.mean = [float(v) for v in m["mean"]]
        p.variance = [float(v) for v in m["variance"]]
        return p
