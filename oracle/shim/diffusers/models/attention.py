import torch


def _chunked_feed_forward(ff, hidden_states, chunk_dim, chunk_size):
    if hidden_states.shape[chunk_dim] % chunk_size != 0:
        raise ValueError("hidden_states dimension must be divisible by chunk_size")
    num_chunks = hidden_states.shape[chunk_dim] // chunk_size
    return torch.cat([ff(c) for c in hidden_states.chunk(num_chunks, dim=chunk_dim)], dim=chunk_dim)
