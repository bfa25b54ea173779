"""flame_amd: MI355X-native server-side aggregation path for cisco-open/flame."""
__version__ = "0.1.0"
