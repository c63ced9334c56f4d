"""ORACLE — test infrastructure only (see lte_oracle.py).  The product package
never imports this."""
