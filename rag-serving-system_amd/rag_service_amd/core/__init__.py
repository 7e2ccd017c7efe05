"""Mirror of the reference's rag_service/core package (retrieval hot path only)."""
