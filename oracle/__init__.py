"""oracle -- TEST INFRASTRUCTURE ONLY: CPU checkers for the gfx950 codec (see oracle/oracle.py)."""
