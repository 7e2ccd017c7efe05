"""MI355X-native drop-in for the retrieval hot path of ngray0/RAG-Serving-System.

Import path: put ``<repo>/rag-serving-system_amd`` on ``sys.path`` and use
``from rag_service_amd.core.retriever import HipRetriever`` where the reference imports
``from rag_service.core.retriever import CupyRetriever`` (main.py:12, batch_processor.py:11).
"""
from ._lib import (HipRetrievalError, HipRetrievalUnavailable, Index, build, get_unique_id,  # noqa: F401
                   load_library, LIB_PATH, HEADER_PATH, SIGNATURES)

__all__ = ["Index", "build", "load_library", "get_unique_id", "HipRetrievalError", "HipRetrievalUnavailable"]
