"""TEST INFRASTRUCTURE ONLY: CPU restatement of the reference path (checker / cpu_baseline)."""
