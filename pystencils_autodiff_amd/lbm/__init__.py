"""Differentiable lattice Boltzmann time stepping (reference ``pystencils_autodiff.lbm``)."""
from ._autodiff_lbstep import AutoDiffLatticeBoltzmannStep, PdfFieldNotDetectedException, SimulationResultsTensors
from ._method import (LBStencil, create_lb_adjoint_rule, create_lb_update_rule, equilibrium_setter, macroscopic_getter,
                      relaxation_rate_from_magic_number)
from .boundaries import (UBB, AdjointBoundaryCondition, AdjointNoSlip, Boundary, FixedDensity, NoSlip, link_coefficients,
                         link_form, link_program, make_slice)

__all__ = ['AutoDiffLatticeBoltzmannStep', 'PdfFieldNotDetectedException', 'SimulationResultsTensors', 'LBStencil',
           'create_lb_update_rule', 'create_lb_adjoint_rule', 'macroscopic_getter', 'equilibrium_setter', 'Boundary',
           'NoSlip', 'UBB', 'FixedDensity', 'AdjointNoSlip', 'AdjointBoundaryCondition', 'link_coefficients', 'link_form',
           'link_program', 'make_slice',
           'relaxation_rate_from_magic_number']
