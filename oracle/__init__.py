"""CPU oracle of the reference hot path -- TEST INFRASTRUCTURE ONLY (see dcor_oracle.h).

Parity status: unpinned (no R, no reference fixtures)."""
