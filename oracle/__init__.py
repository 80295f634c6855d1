"""CPU oracle for the noble-gas CE + RTD-convolution log-likelihood path.

TEST INFRASTRUCTURE ONLY.  Nothing under ``oracle/`` is part of the product: only
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
it, and only as the checker (or the timed CPU baseline) -- never as a fallback for the
HIP path.  The package ``noblegas_rtd_mcmc_amd`` never imports it.

It is a NumPy restatement of the reference's arithmetic (uz226/NobleGas_RTD_MCMC):

* ``oracle.ce``    -- utils/noble_gas_utils.py (atm_std, noble_gas_fun, J_flux)
* ``oracle.rtd``   -- utils/convolution_integral_utils.py (tracer_conv_integral) and the
                      ForwardMod composition of age_ens_runs_mcmc/run_age_mcmc_utils.py:81-163
* ``oracle.stats`` -- PyMC3 3.11.2 StudentT / Beta / Normal / Uniform / HalfNormal logp
                      (third-party, not in the reference; pinned to scipy.stats in tests)
* ``oracle.models``-- the CE model (ng_interp/noble_gas_mcmc.py:184-267), the RTD model
                      (run_age_mcmc_utils.py:275-397) and the joint model, per walker.

Parity pinning: ``tests/golden/make_golden.py`` imports the reference's own
``noble_gas_utils`` / ``convolution_integral_utils`` in the build container and freezes
their outputs as fixtures under ``tests/golden``; ``tests/test_oracle_golden.py`` checks
this restatement against them.  PyMC3 transformed-space Jacobians and DEMetropolisZ are
not installed anywhere here: those pieces are "parity unpinned" (see DESIGN.md).
"""
