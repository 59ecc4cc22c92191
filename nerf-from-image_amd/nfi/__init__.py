"""nfi — MI355X-native volume renderer for the SDF-NeRF inversion loop of
yuliangguo/nerf-from-image (drop-in for run.py:176-350).  See DESIGN.md."""

from .render import (RenderConfig, TriplaneField, configure, field_from_generator, get_config, render,  # noqa: F401
                     render_zbuffer)
from . import ops  # noqa: F401

__all__ = ['render', 'render_zbuffer', 'configure', 'get_config', 'RenderConfig', 'TriplaneField', 'field_from_generator', 'ops']
