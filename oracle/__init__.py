"""TEST INFRASTRUCTURE: CPU restatement of the reference decode path (see pq_oracle.cpp)."""
