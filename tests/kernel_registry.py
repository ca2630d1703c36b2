"""Which rollout-kernel template instantiations the GPU suite has compared against the oracle
in this pytest session (filled by tests/test_gpu_parity.py, checked by
tests/test_gpu_ycoverage.py): a kernel the bench times must be one the suite has run."""

COVERED = {}      # instantiation, e.g. "rollout_wide3_kernel<u64,1,false>" -> [case, ...]


def record_rollout_kernel(name, case):
    COVERED.setdefault(name, []).append(case)
