"""CPU oracle package (test infrastructure only; see hmc_oracle.py header)."""
