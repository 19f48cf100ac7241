"""CPU parity oracle -- TEST INFRASTRUCTURE ONLY (see gsr_oracle.c).  Never imported by the product."""
