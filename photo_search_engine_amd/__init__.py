"""photo_search_engine_amd -- MI355X-native exact flat k-NN backend for Photo_Search_Engine.

The one hot path of the reference (``VectorStore.add_item`` / ``VectorStore.search`` over faiss
IndexFlat, /root/reference/utils/vector_store.py) rebuilt as a C-ABI HIP library (``libvs.so``,
include/vs.h) for gfx950, with the reference's Python surface on top.

    from photo_search_engine_amd.vector_store import VectorStore   # drop-in
    from photo_search_engine_amd.index import FlatIndex            # faiss-IndexFlat-like handle
"""
__version__ = "0.1.0"

__all__ = ["VectorStore", "FlatIndex", "__version__"]


def __getattr__(name):  # lazy: importing the package must not require a GPU
    if name == "VectorStore":
        from .vector_store import VectorStore
        return VectorStore
    if name == "FlatIndex":
        from .index import FlatIndex
        return FlatIndex
    raise AttributeError(name)
