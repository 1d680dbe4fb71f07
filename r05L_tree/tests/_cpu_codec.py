"""Test-only alias: the oracle-backed codec lives in oracle/cpu_codec.py."""
from oracle.cpu_codec import OracleCodec  # noqa: F401
