"""Typed configuration objects of the boosted decoder's constructor API
(reference: src/boosted_neural_ldpc_decoder/struct/)."""
