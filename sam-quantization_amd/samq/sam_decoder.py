"""SAM prompt encoder + mask decoder and the predictor plumbing (f1).

Small compute next to the encoder (~0.1 % of the FLOPs of one prompt round), so plain torch on the
encoder's device.  Parameter names follow the reference so a SAM ``state_dict`` loads unchanged:
``PromptEncoder`` (``segment_anything/modeling/prompt_encoder.py:16-215``), ``MaskDecoder`` +
``MLP`` (``mask_decoder.py:16-178``), ``TwoWayTransformer`` / ``TwoWayAttentionBlock`` /
``Attention`` (``transformer.py:16-240``), ``ResizeLongestSide``
(``segment_anything/utils/transforms.py:16-103``) and ``SamPredictor``
(``segment_anything/predictor.py:17-270``).  Used to report mask IoU between masks predicted from
our encoder's embeddings and from the reference's (north-star parity report).
"""
from __future__ import annotations

import math
from typing import List, Optional, Tuple, Type

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from .modeling import LayerNorm2d, MLPBlock


# ----------------------------------------------------------------------------- prompt encoder
class PositionEmbeddingRandom(nn.Module):
    """Fourier features of (x, y) in [0, 1]^2 through a fixed Gaussian matrix (``:168-215``)."""

    def __init__(self, num_pos_feats: int = 64, scale: Optional[float] = None):
        super().__init__()
        scale = 1.0 if scale is None or scale <= 0.0 else scale
        self.register_buffer("positional_encoding_gaussian_matrix", scale * torch.randn((2, num_pos_feats)))

    def _encode(self, xy01: torch.Tensor) -> torch.Tensor:
        proj = (2.0 * xy01 - 1.0) @ self.positional_encoding_gaussian_matrix.float()
        proj = (2.0 * np.pi) * proj
        return torch.cat([proj.sin(), proj.cos()], dim=-1)

    def forward(self, size: Tuple[int, int]) -> torch.Tensor:
        h, w = size
        dev = self.positional_encoding_gaussian_matrix.device
        ys = (torch.arange(h, device=dev, dtype=torch.float32) + 0.5) / h
        xs = (torch.arange(w, device=dev, dtype=torch.float32) + 0.5) / w
        grid = torch.stack([xs[None, :].expand(h, w), ys[:, None].expand(h, w)], dim=-1)
        return self._encode(grid).to(self.positional_encoding_gaussian_matrix.dtype).permute(2, 0, 1)

    def forward_with_coords(self, coords: torch.Tensor, image_size: Tuple[int, int]) -> torch.Tensor:
        xy = coords.clone().float()
        xy[..., 0] = xy[..., 0] / image_size[1]
        xy[..., 1] = xy[..., 1] / image_size[0]
        return self._encode(xy).to(coords.dtype)


class PromptEncoder(nn.Module):
    def __init__(self, embed_dim: int, image_embedding_size: Tuple[int, int], input_image_size: Tuple[int, int],
                 mask_in_chans: int, activation: Type[nn.Module] = nn.GELU):
        super().__init__()
        self.embed_dim = embed_dim
        self.input_image_size = input_image_size
        self.image_embedding_size = image_embedding_size
        self.pe_layer = PositionEmbeddingRandom(embed_dim // 2)
        self.num_point_embeddings = 4          # negative / positive point, box corner 1 / 2
        self.point_embeddings = nn.ModuleList([nn.Embedding(1, embed_dim) for _ in range(4)])
        self.not_a_point_embed = nn.Embedding(1, embed_dim)
        self.mask_input_size = (4 * image_embedding_size[0], 4 * image_embedding_size[1])
        self.mask_downscaling = nn.Sequential(
            nn.Conv2d(1, mask_in_chans // 4, kernel_size=2, stride=2), LayerNorm2d(mask_in_chans // 4), activation(),
            nn.Conv2d(mask_in_chans // 4, mask_in_chans, kernel_size=2, stride=2), LayerNorm2d(mask_in_chans),
            activation(), nn.Conv2d(mask_in_chans, embed_dim, kernel_size=1))
        self.no_mask_embed = nn.Embedding(1, embed_dim)

    def get_dense_pe(self) -> torch.Tensor:
        return self.pe_layer(self.image_embedding_size).unsqueeze(0)

    def _points(self, coords, labels, pad: bool):
        coords = coords + 0.5
        if pad:
            b = coords.shape[0]
            coords = torch.cat([coords, coords.new_zeros((b, 1, 2))], dim=1)
            labels = torch.cat([labels, -labels.new_ones((b, 1))], dim=1)
        emb = self.pe_layer.forward_with_coords(coords, self.input_image_size)
        pad_mask = (labels == -1)[..., None]
        emb = torch.where(pad_mask, self.not_a_point_embed.weight.expand_as(emb), emb)
        emb = emb + (labels == 0)[..., None] * self.point_embeddings[0].weight
        emb = emb + (labels == 1)[..., None] * self.point_embeddings[1].weight
        return emb

    def _boxes(self, boxes):
        corners = self.pe_layer.forward_with_coords((boxes + 0.5).reshape(-1, 2, 2), self.input_image_size)
        return torch.stack([corners[:, 0] + self.point_embeddings[2].weight[0],
                            corners[:, 1] + self.point_embeddings[3].weight[0]], dim=1)

    def forward(self, points: Optional[Tuple[torch.Tensor, torch.Tensor]], boxes: Optional[torch.Tensor],
                masks: Optional[torch.Tensor]):
        if points is not None:
            bs = points[0].shape[0]
        elif boxes is not None:
            bs = boxes.shape[0]
        elif masks is not None:
            bs = masks.shape[0]
        else:
            bs = 1
        dev = self.point_embeddings[0].weight.device
        parts = [torch.empty((bs, 0, self.embed_dim), device=dev)]
        if points is not None:
            parts.append(self._points(points[0], points[1], pad=boxes is None))
        if boxes is not None:
            parts.append(self._boxes(boxes))
        sparse = torch.cat(parts, dim=1)
        if masks is not None:
            dense = self.mask_downscaling(masks)
        else:
            dense = self.no_mask_embed.weight.to(sparse.dtype).reshape(1, -1, 1, 1).expand(
                bs, -1, self.image_embedding_size[0], self.image_embedding_size[1])
        return sparse, dense


# ----------------------------------------------------------------------------- two-way transformer
class Attention(nn.Module):
    """Multi-head attention whose projections may shrink the width by ``downsample_rate``."""

    def __init__(self, embedding_dim: int, num_heads: int, downsample_rate: int = 1):
        super().__init__()
        self.embedding_dim = embedding_dim
        self.internal_dim = embedding_dim // downsample_rate
        self.num_heads = num_heads
        assert self.internal_dim % num_heads == 0, "num_heads must divide embedding_dim."
        self.q_proj = nn.Linear(embedding_dim, self.internal_dim)
        self.k_proj = nn.Linear(embedding_dim, self.internal_dim)
        self.v_proj = nn.Linear(embedding_dim, self.internal_dim)
        self.out_proj = nn.Linear(self.internal_dim, embedding_dim)

    def forward(self, q: torch.Tensor, k: torch.Tensor, v: torch.Tensor) -> torch.Tensor:
        h = self.num_heads

        def split(t):
            b, n, c = t.shape
            return t.view(b, n, h, c // h).transpose(1, 2)

        qh, kh, vh = split(self.q_proj(q)), split(self.k_proj(k)), split(self.v_proj(v))
        att = torch.softmax((qh @ kh.transpose(-1, -2)) / math.sqrt(qh.shape[-1]), dim=-1)
        o = (att @ vh).transpose(1, 2)
        return self.out_proj(o.reshape(o.shape[0], o.shape[1], -1))


class TwoWayAttentionBlock(nn.Module):
    def __init__(self, embedding_dim: int, num_heads: int, mlp_dim: int = 2048,
                 activation: Type[nn.Module] = nn.ReLU, attention_downsample_rate: int = 2,
                 skip_first_layer_pe: bool = False):
        super().__init__()
        self.self_attn = Attention(embedding_dim, num_heads)
        self.norm1 = nn.LayerNorm(embedding_dim)
        self.cross_attn_token_to_image = Attention(embedding_dim, num_heads, attention_downsample_rate)
        self.norm2 = nn.LayerNorm(embedding_dim)
        self.mlp = MLPBlock(embedding_dim, mlp_dim, activation)
        self.norm3 = nn.LayerNorm(embedding_dim)
        self.norm4 = nn.LayerNorm(embedding_dim)
        self.cross_attn_image_to_token = Attention(embedding_dim, num_heads, attention_downsample_rate)
        self.skip_first_layer_pe = skip_first_layer_pe

    def forward(self, queries, keys, query_pe, key_pe):
        if self.skip_first_layer_pe:
            queries = self.self_attn(queries, queries, queries)
        else:
            qp = queries + query_pe
            queries = queries + self.self_attn(qp, qp, queries)
        queries = self.norm1(queries)
        kp = keys + key_pe
        queries = self.norm2(queries + self.cross_attn_token_to_image(queries + query_pe, kp, keys))
        queries = self.norm3(queries + self.mlp(queries))
        keys = self.norm4(keys + self.cross_attn_image_to_token(kp, queries + query_pe, queries))
        return queries, keys


class TwoWayTransformer(nn.Module):
    def __init__(self, depth: int, embedding_dim: int, num_heads: int, mlp_dim: int,
                 activation: Type[nn.Module] = nn.ReLU, attention_downsample_rate: int = 2):
        super().__init__()
        self.depth, self.embedding_dim, self.num_heads, self.mlp_dim = depth, embedding_dim, num_heads, mlp_dim
        self.layers = nn.ModuleList([
            TwoWayAttentionBlock(embedding_dim, num_heads, mlp_dim, activation, attention_downsample_rate,
                                 skip_first_layer_pe=(i == 0)) for i in range(depth)])
        self.final_attn_token_to_image = Attention(embedding_dim, num_heads, attention_downsample_rate)
        self.norm_final_attn = nn.LayerNorm(embedding_dim)

    def forward(self, image_embedding, image_pe, point_embedding):
        keys = image_embedding.flatten(2).transpose(1, 2)
        key_pe = image_pe.flatten(2).transpose(1, 2)
        queries = point_embedding
        for layer in self.layers:
            queries, keys = layer(queries, keys, point_embedding, key_pe)
        att = self.final_attn_token_to_image(queries + point_embedding, keys + key_pe, keys)
        return self.norm_final_attn(queries + att), keys


# ----------------------------------------------------------------------------- mask decoder
class MLP(nn.Module):
    def __init__(self, input_dim: int, hidden_dim: int, output_dim: int, num_layers: int,
                 sigmoid_output: bool = False):
        super().__init__()
        self.num_layers = num_layers
        dims = [input_dim] + [hidden_dim] * (num_layers - 1) + [output_dim]
        self.layers = nn.ModuleList(nn.Linear(a, b) for a, b in zip(dims[:-1], dims[1:]))
        self.sigmoid_output = sigmoid_output

    def forward(self, x):
        for i, layer in enumerate(self.layers):
            x = layer(x)
            if i + 1 < self.num_layers:
                x = F.relu(x)
        return torch.sigmoid(x) if self.sigmoid_output else x


class MaskDecoder(nn.Module):
    def __init__(self, *, transformer_dim: int, transformer: nn.Module, num_multimask_outputs: int = 3,
                 activation: Type[nn.Module] = nn.GELU, iou_head_depth: int = 3, iou_head_hidden_dim: int = 256):
        super().__init__()
        self.transformer_dim = transformer_dim
        self.transformer = transformer
        self.num_multimask_outputs = num_multimask_outputs
        self.iou_token = nn.Embedding(1, transformer_dim)
        self.num_mask_tokens = num_multimask_outputs + 1
        self.mask_tokens = nn.Embedding(self.num_mask_tokens, transformer_dim)
        c4, c8 = transformer_dim // 4, transformer_dim // 8
        self.output_upscaling = nn.Sequential(
            nn.ConvTranspose2d(transformer_dim, c4, kernel_size=2, stride=2), LayerNorm2d(c4), activation(),
            nn.ConvTranspose2d(c4, c8, kernel_size=2, stride=2), activation())
        self.output_hypernetworks_mlps = nn.ModuleList(
            [MLP(transformer_dim, transformer_dim, c8, 3) for _ in range(self.num_mask_tokens)])
        self.iou_prediction_head = MLP(transformer_dim, iou_head_hidden_dim, self.num_mask_tokens, iou_head_depth)

    def predict_masks(self, image_embeddings, image_pe, sparse_prompt_embeddings, dense_prompt_embeddings):
        dt = image_embeddings.dtype
        sparse = sparse_prompt_embeddings.to(dt)
        out_tokens = torch.cat([self.iou_token.weight, self.mask_tokens.weight], dim=0)
        tokens = torch.cat([out_tokens[None].expand(sparse.shape[0], -1, -1), sparse], dim=1)
        n = tokens.shape[0]
        src = image_embeddings.repeat_interleave(n, dim=0) + dense_prompt_embeddings.to(dt)
        pos = image_pe.repeat_interleave(n, dim=0)
        b, c, h, w = src.shape
        hs, src = self.transformer(src, pos, tokens)
        up = self.output_upscaling(src.transpose(1, 2).reshape(b, c, h, w))
        hyper = torch.stack([mlp(hs[:, 1 + i]) for i, mlp in enumerate(self.output_hypernetworks_mlps)], dim=1)
        bu, cu, hu, wu = up.shape
        masks = (hyper @ up.view(bu, cu, hu * wu)).view(bu, -1, hu, wu)
        return masks, self.iou_prediction_head(hs[:, 0])

    def forward(self, image_embeddings, image_pe, sparse_prompt_embeddings, dense_prompt_embeddings,
                multimask_output: bool):
        masks, iou = self.predict_masks(image_embeddings, image_pe, sparse_prompt_embeddings, dense_prompt_embeddings)
        sl = slice(1, None) if multimask_output else slice(0, 1)
        return masks[:, sl], iou[:, sl]


def build_prompt_decoder(prompt_embed_dim: int = 256, image_size: int = 1024, patch: int = 16):
    """The reference's prompt encoder / mask decoder hyper-parameters (``build_sam.py:55-107``)."""
    emb = image_size // patch
    pe = PromptEncoder(embed_dim=prompt_embed_dim, image_embedding_size=(emb, emb),
                       input_image_size=(image_size, image_size), mask_in_chans=16)
    md = MaskDecoder(num_multimask_outputs=3, transformer_dim=prompt_embed_dim, iou_head_depth=3,
                     iou_head_hidden_dim=256,
                     transformer=TwoWayTransformer(depth=2, embedding_dim=prompt_embed_dim, mlp_dim=2048, num_heads=8))
    return pe, md


def postprocess_masks(masks: torch.Tensor, img_size: int, input_size, original_size) -> torch.Tensor:
    """``Sam.postprocess_masks`` (``sam.py:133-162``): upsample to the padded input, crop, resize."""
    m = F.interpolate(masks, (img_size, img_size), mode="bilinear", align_corners=False)
    m = m[..., : input_size[0], : input_size[1]]
    return F.interpolate(m, tuple(original_size), mode="bilinear", align_corners=False)


def mask_iou(a: torch.Tensor, b: torch.Tensor) -> float:
    """Intersection over union of two boolean masks (``script/evaluation2.py`` get_iou)."""
    a, b = a.bool(), b.bool()
    union = (a | b).sum().item()
    return 1.0 if union == 0 else (a & b).sum().item() / union


# ----------------------------------------------------------------------------- predictor plumbing
class ResizeLongestSide:
    """Resize so the longest side equals ``target_length`` (``utils/transforms.py:16-103``)."""

    def __init__(self, target_length: int):
        self.target_length = target_length

    @staticmethod
    def get_preprocess_shape(oldh: int, oldw: int, long_side_length: int) -> Tuple[int, int]:
        scale = long_side_length * 1.0 / max(oldh, oldw)
        return int(oldh * scale + 0.5), int(oldw * scale + 0.5)

    def apply_image(self, image: np.ndarray) -> np.ndarray:
        h, w = self.get_preprocess_shape(image.shape[0], image.shape[1], self.target_length)
        if (h, w) == image.shape[:2]:
            return image
        from PIL import Image
        return np.array(Image.fromarray(image).resize((w, h), Image.BILINEAR))

    def apply_coords(self, coords: np.ndarray, original_size) -> np.ndarray:
        oh, ow = original_size
        nh, nw = self.get_preprocess_shape(oh, ow, self.target_length)
        c = np.array(coords, dtype=float, copy=True)
        c[..., 0] *= nw / ow
        c[..., 1] *= nh / oh
        return c

    def apply_boxes(self, boxes: np.ndarray, original_size) -> np.ndarray:
        return self.apply_coords(np.asarray(boxes).reshape(-1, 2, 2), original_size).reshape(-1, 4)

    def apply_coords_torch(self, coords: torch.Tensor, original_size) -> torch.Tensor:
        oh, ow = original_size
        nh, nw = self.get_preprocess_shape(oh, ow, self.target_length)
        c = coords.clone().to(torch.float)
        c[..., 0] = c[..., 0] * (nw / ow)
        c[..., 1] = c[..., 1] * (nh / oh)
        return c


class SamPredictor:
    """Embed an image once with the (quantized, HIP) encoder, then predict masks for prompts
    (``segment_anything/predictor.py``: ``set_image`` / ``set_torch_image`` / ``predict`` /
    ``predict_torch`` / ``get_image_embedding`` / ``reset_image``)."""

    def __init__(self, sam_model):
        self.model = sam_model
        self.transform = ResizeLongestSide(sam_model.image_encoder.img_size)
        self.reset_image()

    @property
    def device(self) -> torch.device:
        return self.model.device

    def reset_image(self) -> None:
        self.is_image_set = False
        self.features = None
        self.orig_h = self.orig_w = self.input_h = self.input_w = None

    def set_image(self, image: np.ndarray, image_format: str = "RGB") -> None:
        assert image_format in ("RGB", "BGR"), f"image_format must be in ['RGB', 'BGR'], is {image_format}."
        if image_format != self.model.image_format:
            image = image[..., ::-1]
        inp = self.transform.apply_image(np.ascontiguousarray(image))
        t = torch.as_tensor(inp, device=self.device).permute(2, 0, 1).contiguous()[None]
        self.set_torch_image(t, image.shape[:2])

    @torch.no_grad()
    def set_torch_image(self, transformed_image: torch.Tensor, original_image_size) -> None:
        assert (transformed_image.dim() == 4 and transformed_image.shape[1] == 3
                and max(*transformed_image.shape[2:]) == self.model.image_encoder.img_size), \
            f"set_torch_image input must be BCHW with long side {self.model.image_encoder.img_size}."
        self.reset_image()
        self.original_size = tuple(original_image_size)
        self.input_size = tuple(transformed_image.shape[-2:])
        enc = self.model.image_encoder
        # only the GPTQ encoder (samq.modeling) has the uint8 patch-embedding entry; any other
        # encoder (e.g. the fq_vit W8A8 one, which has no ``is_quantized``) takes preprocess + forward
        fused_u8 = getattr(enc, "is_quantized", None)
        if transformed_image.is_cuda and transformed_image.dtype == torch.uint8 and fused_u8 is not None and fused_u8():
            # HIP engine: Sam.preprocess (normalise + zero-pad) runs inside the patch embedding
            # kernel on the raw uint8 pixels (samq_patch_embed_u8)
            self.features = enc.engine()(transformed_image.contiguous(), out_dtype=torch.float32,
                                         pixel_norm=(self.model.pixel_mean, self.model.pixel_std))
        else:
            x = self.model.preprocess(transformed_image.float())
            p = next(enc.parameters(), None)
            dt = p.dtype if p is not None and p.is_floating_point() else torch.float32
            self.features = enc(x.to(dt)).float()
        self.is_image_set = True

    def get_image_embedding(self) -> torch.Tensor:
        if not self.is_image_set:
            raise RuntimeError("An image must be set with .set_image(...) to generate an embedding.")
        return self.features

    @torch.no_grad()
    def predict_torch(self, point_coords, point_labels, boxes=None, mask_input=None, multimask_output=True,
                      return_logits=False):
        if not self.is_image_set:
            raise RuntimeError("An image must be set with .set_image(...) before mask prediction.")
        points = (point_coords, point_labels) if point_coords is not None else None
        sparse, dense = self.model.prompt_encoder(points=points, boxes=boxes, masks=mask_input)
        low, iou = self.model.mask_decoder(self.features, self.model.prompt_encoder.get_dense_pe(), sparse, dense,
                                           multimask_output)
        masks = postprocess_masks(low, self.model.image_encoder.img_size, self.input_size, self.original_size)
        if not return_logits:
            masks = masks > self.model.mask_threshold
        return masks, iou, low

    def predict(self, point_coords=None, point_labels=None, box=None, mask_input=None, multimask_output=True,
                return_logits=False):
        if not self.is_image_set:
            raise RuntimeError("An image must be set with .set_image(...) before mask prediction.")
        dev = self.device
        pc = pl = bx = mi = None
        if point_coords is not None:
            assert point_labels is not None, "point_labels must be supplied if point_coords is supplied."
            pc = torch.as_tensor(self.transform.apply_coords(point_coords, self.original_size), dtype=torch.float,
                                 device=dev)[None]
            pl = torch.as_tensor(point_labels, dtype=torch.int, device=dev)[None]
        if box is not None:
            bx = torch.as_tensor(self.transform.apply_boxes(box, self.original_size), dtype=torch.float,
                                 device=dev)[None]
        if mask_input is not None:
            mi = torch.as_tensor(mask_input, dtype=torch.float, device=dev)[None]
        masks, iou, low = self.predict_torch(pc, pl, bx, mi, multimask_output, return_logits)
        return masks[0].cpu().numpy(), iou[0].cpu().numpy(), low[0].cpu().numpy()
