"""Parameter shape lists of the reference's models, in `model.parameters()`
order.  The strategy step only sees these shapes; the bench
and tests build synthetic arenas from them without instantiating the models.

gpt2(...)  example/nanogpt/nanogpt.py GPT: wte [V,C] (tied with lm_head, so
           listed once), wpe [1024,C], per block ln_1 w/b, c_attn w [3C,C] b,
           attn.c_proj w [C,C] b, ln_2 w/b, c_fc w [4C,C] b, mlp.c_proj w [C,4C] b,
           then ln_f w/b.  Sizes: GPTConfig.gpt2_small/base/medium (:160-171).
mnist_cnn  example/mnist.py CNN (:31-63): 4 conv+BN blocks, 2 linear layers.
"""

GPT2_SIZES = {
    "small": dict(n_layer=4, n_embd=128),    # char-level default
    "base": dict(n_layer=12, n_embd=768),    # GPT-2 124M
    "medium": dict(n_layer=24, n_embd=1024),  # GPT-2 350M
    "large": dict(n_layer=36, n_embd=1280),
    "xl": dict(n_layer=48, n_embd=1600),
}


def gpt2(size="base", vocab_size=50304, block_size=1024, bias=True):
    cfg = GPT2_SIZES[size]
    L, C = cfg["n_layer"], cfg["n_embd"]
    shapes = [(vocab_size, C), (block_size, C)]
    for _ in range(L):
        blk = [(C,), (C,), (3 * C, C), (3 * C,), (C, C), (C,), (C,), (C,), (4 * C, C), (4 * C,), (C, 4 * C), (C,)]
        if not bias:
            blk = [s for s, is_bias in zip(blk, [0, 1, 0, 1, 0, 1, 0, 1, 0, 1, 0, 1]) if not is_bias]
        shapes += blk
    shapes += [(C,), (C,)] if bias else [(C,)]
    return shapes


def mnist_cnn():
    shapes = []
    for cin, cout in ((1, 64), (64, 64), (64, 128), (128, 128)):
        shapes += [(cout, cin, 3, 3), (cout,), (cout,), (cout,)]  # conv w, conv b, bn w, bn b
    shapes += [(256, 128 * 7 * 7), (256,), (10, 256), (10,)]
    return shapes


MODELS = {
    "gpt2-124m": lambda: gpt2("base"),
    "gpt2-350m": lambda: gpt2("medium"),
    "gpt2-char": lambda: gpt2("small", vocab_size=66),
    "mnist-cnn": mnist_cnn,
}


def numel(shapes):
    n = 0
    for s in shapes:
        k = 1
        for d in s:
            k *= d
        n += k
    return n
