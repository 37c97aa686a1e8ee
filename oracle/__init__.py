"""CPU oracle (test infrastructure only -- see ref_cpu.py's header)."""
