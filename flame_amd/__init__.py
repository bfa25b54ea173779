"""flame_amd: MI355X-native server-side aggregation path for cisco-open/flame.

Drop-in replacements for flame's FedAvg / FedAdam / FedYogi / FedAdaGrad /
FedBuff server optimizers (``flame_amd.optimizer``), backed by hand-written
gfx950 HIP kernels behind the C ABI in ``include/flame_amd.h``.
``flame_amd.optimizers.install()`` registers them into flame's own
``optimizer_provider``.
"""
__version__ = "0.1.0"
