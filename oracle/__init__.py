"""CPU oracle (test infrastructure only).  See oracle/ldpc_oracle.py."""
