"""Drop-in replacement of the reference's `FEANet` package (longfish/Multigrid-FEANet/FEANet):
same module names, classes and signatures; the operators run as HIP kernels on the MI355X
(feanet_amd.ops).  Put `multigrid-feanet_amd/` first on sys.path and create tensors on the
HIP device (e.g. `torch.set_default_device('cuda')`); CPU tensors raise instead of silently
falling back.  See INTEGRATION.md."""
