"""CPU oracle — test infrastructure only (see oracle/hstu_oracle.py header)."""
