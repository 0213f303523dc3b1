"""MI355X-native Gibbs/MH sampler for the Abe (2009/2015) hierarchical Pareto/NBD model.

Drop-in for lucagem29/mcmc_clv_model's sampler entry points:

    from mcmc_clv_model_amd import mcmc_draw_parameters        # src/models/bivariate/mcmc.py:437
    from mcmc_clv_model_amd import mcmc_draw_parameters_rfm_m  # src/models/trivariate/mcmc.py:580

Posterior analysis: draw_future_transactions (bi:506 / tri:660), the Table 4 helpers
of utils/analysis_bi_helpers.py and the weekly tracking curve, also on the GPU (analysis.py).

The per-sweep work runs in hand-written HIP kernels for gfx950 (csrc/), bound through the C
ABI in include/clvmcmc.h.  There is no CPU fallback.
"""
from .analysis import (chain_total_loglik, compute_table4, draw_future_transactions,
                       draw_future_transactions_rfm_m, post_mean_lambdas, post_mean_mus,
                       posterior_weekly_tracking)
from .bivariate import mcmc_draw_parameters
from .trivariate import mcmc_draw_parameters_rfm_m

__all__ = ["mcmc_draw_parameters", "mcmc_draw_parameters_rfm_m", "draw_future_transactions",
           "draw_future_transactions_rfm_m", "post_mean_lambdas", "post_mean_mus", "chain_total_loglik",
           "compute_table4", "posterior_weekly_tracking"]
__version__ = "0.1.0"
