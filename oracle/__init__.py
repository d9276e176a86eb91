"""ORACLE -- test infrastructure (CPU restatement of the reference's hot
path).  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may
import it; the cubed_amd package never does."""
