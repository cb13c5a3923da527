"""ORACLE — CPU restatement of the reference's Gibbs sweep (test infrastructure only).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this package.  The product path (hmsc_amd) never does.
"""
