"""MI355X-native drop-in for the ``nightcore_analyzer`` package (placeholder; filled in below)."""
__version__ = "0.3.0"
