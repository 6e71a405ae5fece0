"""sparc_ldpc_amd — MI355X (gfx950) SPARC AMP decoder with its LDPC outer code.

Drop-in for the AMP hot path of Spimp/sparc_ldpc (ldpc/sparc_ldpc.py:14-222,
ldpc/amp_test.py:14-50): the same names, argument order and return shapes,
with the design operator and the whole iteration loop running as HIP kernels
in ``libsparc_amp.so`` (C ABI: include/sparc_amp.h).  There is no CPU
fallback: without the library or a HIP device every call raises.
"""
from ._lib import SparcAmpError, load as load_library
from .operators import (SparcOperator, AbOp, AzOp, make_ordering, sub_fht, block_sub_fht, dense_transforms,
                        gaussian_transforms,
                        sparc_transforms, sparc_transforms_shorter, default_device)
from .amp import amp, amp_test, amp_batch, operator_of
from .harness import (SPARCParams, LDPCParams, pa_parameterised, bits2indices, ber_of,
                      amp_ldpc_sim, mc_decode, mc_decode_batched, mc_stream, draw_reps, ebno_to_sigma, ber_point, waterfall_plain,
                      amp_test_reps, amp_init_test)
from . import ldpc
from .ldpc import code, LdpcBpError
from .joint import (JointDecoder, joint_decoder, soft_amp_ldpc_sim, hardinitbeta_amp_ldpc_sim, sim_ldpc, soft_hard_plot,
                    waterfall, sp2bp, bp2sp, mc_joint)
from . import threshold
from .threshold import (hard_initialisation, prep_y, calc_E, hist_E, calc_I_e, J, J_inverse,
                        soft_amp_ldpc_hardinit, ber_from_LLRs, soft_hardinit_plot, calc_E_batch, amp_exit_curve)
from . import dist

__version__ = "0.1.0"
