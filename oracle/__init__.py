"""CPU oracle (test infrastructure only): see oracle/mapf_oracle.c."""
