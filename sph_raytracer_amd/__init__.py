"""sph_raytracer_amd — MI355X-native spherical-grid raytracer (drop-in for Evidlo/sph_raytracer).

    from sph_raytracer_amd import SphericalGrid, ConeRectGeom, Operator
"""
from .raytracer import Operator
from .geometry import *  # noqa: F401,F403
from .geometry import __all__ as _geometry_all

__all__ = ['Operator'] + list(_geometry_all)
