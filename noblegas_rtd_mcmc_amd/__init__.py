"""MI355X-native log-likelihood engine for the noble-gas CE and RTD-convolution models
of uz226/NobleGas_RTD_MCMC.  The compute path is libngrtd.so (HIP,
gfx950); importing this package does not touch the GPU."""
__version__ = "0.1.0"
