"""Test-only CPU oracle for the Dion data-parallel step (see dion_oracle.py header)."""
