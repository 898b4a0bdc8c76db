"""CPU oracle -- test infrastructure only (see neus_oracle.py)."""
