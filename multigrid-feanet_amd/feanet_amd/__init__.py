"""feanet_amd — MI355X-native geometric-multigrid hot path of longfish/Multigrid-FEANet.

  feanet_amd.ops          tensor-level HIP operators (KNet apply, Jacobi sweep, R, P, norms)
  feanet_amd.solver       MultigridSolver: fused-kernel V-cycle over framed level buffers
  feanet_amd.mesh_setup   vectorised discretisation tables (pattern maps, stencils)
  FEANet.*                drop-in modules with the reference's names (sibling package)
"""
from . import mesh_setup  # noqa: F401


def __getattr__(name):
    # lazy: importing the package must not require the HIP library (CPU-only test collection)
    if name == "MultigridSolver":
        from .solver import MultigridSolver
        return MultigridSolver
    if name in ("ops", "solver", "_lib"):
        import importlib
        return importlib.import_module(f".{name}", __name__)
    raise AttributeError(name)
