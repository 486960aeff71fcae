"""ORACLE -- TEST INFRASTRUCTURE ONLY (CPU restatement of the reference; see flinkwin_oracle.cpp)."""
