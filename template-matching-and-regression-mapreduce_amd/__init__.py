"""tmr_amd: MI355X-native TMR hot path (placeholder, filled in below)."""
from . import synth  # noqa: F401
