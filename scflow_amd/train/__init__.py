"""Training step of the SCFlow refinement path: autograd Functions with
HIP forward and backward kernels (``functions``)."""
