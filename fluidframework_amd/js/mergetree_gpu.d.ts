/*
 * mergetree_gpu.d.ts — typings of the JavaScript facade over the MI355X replay engine
 * (mergetree_gpu.js -> mt_napi.node -> libmtreplay.so, include/mt_engine.h). Names and argument meaning
 * follow the reference merge-tree Client (packages/dds/merge-tree/src/client.ts) and MergeTree
 * (mergeTree.ts) surfaces the facade mirrors; TypeScript callers of @fluidframework/merge-tree switch by
 * replacing `Client` with `ReplayEngine.client(doc)`.
 */

/** MergeTreeDeltaType values of IMergeTreeOp.type (ops.ts:29-34) plus the non-op message */
export declare const OP: { readonly INSERT: 0; readonly REMOVE: 1; readonly ANNOTATE: 2; readonly GROUP: 3; readonly NOOP: 4 };
/** ReferenceType values the engine models for local references (ops.ts) */
export declare const ReferenceType: { readonly Simple: 0; readonly SlideOnRemove: 0x40 };
/** constants.ts */
export declare const LocalClientId: -1;
export declare const UnassignedSequenceNumber: -1;

/** include/mt_engine.h mt_caps (per-document capacities; promotion grows documents past them) */
export interface Caps {
    ncap: number; hcap: number; acap: number; mcap: number; gcap: number; ccap: number;
    /** delta event log words per document (0: no delta events) */
    dcap?: number;
    /** local references per document (0: none) */
    rcap?: number;
    /** PermutationVector handles per document (0: no HandleTable) */
    pcap?: number;
}
export declare const DEFAULT_CAPS: Caps;

export type PropertySet = { [key: string]: unknown };
export interface ICombiningOp { name: "rewrite" }
/** a segment spec: a string, {text, props}, or a marker {marker: {refType}, props} */
export type SegmentSpec = string | { text: string; props?: PropertySet } | { marker: { refType: number }; props?: PropertySet };

/** IRelativePosition (ops.ts:56-61): a position before / after the marker whose "markerId" is id */
export interface IRelativePosition { id: string; before?: boolean; offset?: number }

/** IMergeTreeOp (ops.ts:63-102) as the facade sends and receives it; a sequenced op may name its positions
 * relative to markers instead (engines with caps.dcap or caps.rcap > 0) */
export type MergeTreeOp =
    | { type: 0; pos1?: number; relativePos1?: IRelativePosition; seg: SegmentSpec }
    | { type: 1; pos1?: number; pos2?: number; relativePos1?: IRelativePosition; relativePos2?: IRelativePosition }
    | { type: 2; pos1?: number; pos2?: number; relativePos1?: IRelativePosition; relativePos2?: IRelativePosition;
        props: PropertySet; combiningOp?: ICombiningOp }
    | { type: 3; ops: MergeTreeOp[] };

/** ISequencedDocumentMessage fields applyMsg reads (protocol-definitions) */
export interface SequencedMessage {
    clientId: string;
    sequenceNumber: number;
    referenceSequenceNumber: number;
    minimumSequenceNumber: number;
    type: "op" | string;
    contents?: MergeTreeOp;
}

/** a segment handle (mt_seg_ref): the row's stable id and generation, where the position falls in it */
export interface SegmentHandle {
    rid: number; gen: number; offset: number; length: number; seq: number; client: number;
    /** undefined when not removed; -1 = a pending local remove */
    removedSeq: number | undefined; removedClient: number;
    /** the segment's index in walkAllSegments order (its record in the canonical dump) */
    ordinal: number;
}

/** a segment as the reference's ISegment reads (decodeDump / GpuClient.segments()), with its handle and local position */
export interface SegmentObject {
    type: "TextSegment" | "Marker" | "PermutationSegment";
    cachedLength: number; seq: number; clientId: string | -1;
    removedSeq?: number; removedClientId?: string | -1; localSeq?: number; localRemovedSeq?: number;
    properties?: PropertySet; text?: string; refType?: number; start?: number;
    leaf: number; ordinal: number; rid?: number; gen?: number;
    /** position and localNetLength in the local view when read */
    pos?: number; len?: number;
}

export interface DecodedDump {
    currentSeq: number; minSeq: number; localSeq: number; length: number; nleaf: number; localLength?: number;
    segments: SegmentObject[];
}

export interface LocalReferenceHandle { doc: number; index: number }

/** one event of the "sequenceDelta" / "maintenance" stream (include/mt_oplog.h MT_DELTA_*) */
export interface DeltaEvent {
    operation: "INSERT" | "REMOVE" | "ANNOTATE" | "REGEN" | "APPEND" | "SPLIT" | "UNLINK";
    seq: number;
    deltaSegments: Array<{ position?: number; length: number; opType?: number; propertyDeltas?: PropertySet }>;
}

export declare class Interner {
    key(k: string): number;
    value(v: unknown): number;
    /** a SubSequence item's id (the units of a SubSequence row) and back */
    item(v: unknown): number;
    itemObj(i: number): unknown;
}

export declare function decodeDeltas(words: Int32Array, interner: Interner): DeltaEvent[];

/** the canonical segment dump (include/mt_oplog.h) as segment objects; nameOf maps long client indices to ids */
export declare function decodeDump(bytes: Uint8Array, interner: Interner, nameOf: (i: number) => string | -1): DecodedDump;

/** A batch of documents resident in one GPU's HBM; queued events apply at the next read (one launch per read). */
export declare class ReplayEngine {
    constructor(ndocs: number, caps?: Caps, device?: number);
    readonly ndocs: number;
    readonly interner: Interner;
    client(doc: number): GpuClient;
    /** startOrUpdateCollaboration for every document (client.ts:1053-1073): one minSeq / currentSeq, or one per document */
    startCollaboration(localNames: string[], minSeq?: number | ArrayLike<number>, currentSeq?: number | ArrayLike<number>): void;
    /** submit every queued event, replay on the GPU, wait */
    flush(): void;
    /** per-document FNV-1a-64 digests of the canonical segment dump */
    digests(): BigUint64Array;
    longIndex(name: string): number;
}

/** MergeTree-level calls with explicit (refSeq, clientId, seq) (mergeTree.ts:2001-2031, 2598-2738) */
export declare class GpuMergeTree {
    /** one segment per call; clientId: a long client id or LocalClientId; seq UnassignedSequenceNumber = local pending */
    insertSegments(pos: number, segments: [SegmentSpec], refSeq: number, clientId: string | -1, seq: number): void;
    /** overwrite = true is not modelled (throws) */
    markRangeRemoved(start: number, end: number, refSeq: number, clientId: string | -1, seq: number, overwrite?: boolean): void;
    annotateRange(start: number, end: number, props: PropertySet, combiningOp: ICombiningOp | undefined, refSeq: number,
        clientId: string | -1, seq: number): void;
}

/** One replica: the reference Client surface (client.ts:43) */
export declare class GpuClient {
    readonly engine: ReplayEngine;
    readonly doc: number;
    readonly mergeTree: GpuMergeTree;
    readonly longClientId: string | undefined;
    getCurrentSeq(): number;
    /** Client.applyMsg (client.ts:797-819), group ops included */
    applyMsg(msg: SequencedMessage): void;
    insertTextLocal(pos: number, text: string, props?: PropertySet): MergeTreeOp | undefined;
    /** SharedSequence.insert (sequence sharedSequence.ts:116-125): a SubSequence of `items` */
    insertItemsLocal(pos: number, items: unknown[], props?: PropertySet): MergeTreeOp | undefined;
    /** SharedSequence.getItems (sharedSequence.ts:150-183) / getItemCount of a SubSequence document */
    getItems(start: number, end?: number): unknown[];
    getItemCount(): number;
    insertMarkerLocal(pos: number, refType: number, props?: PropertySet): MergeTreeOp;
    removeRangeLocal(start: number, end: number): MergeTreeOp;
    annotateRangeLocal(start: number, end: number, props: PropertySet, combiningOp?: ICombiningOp): MergeTreeOp;
    /** new LocalReference + Client.addLocalReference at getContainingSegment(pos); engines with caps.rcap > 0 */
    createLocalReference(pos: number, refType?: number): LocalReferenceHandle;
    /** LocalReference.toPosition(): -1 detached; throws where the reference's addLocalReference threw */
    localReferencePosition(ref: LocalReferenceHandle): number;
    /** Client.removeLocalReference: the reference leaves its segment's collection (keeps segment and offset) */
    removeLocalReference(ref: LocalReferenceHandle): void;
    insertAtReferencePositionLocal(ref: LocalReferenceHandle, text: string): void;
    /** Client.regeneratePendingOp for every op in flight (engines with caps.dcap > 0) */
    regeneratePendingOps(): Array<{ type: number; pos1: number; length: number }>;
    /** Client.posFromRelativePos in the local view: -1 if no marker holds the id */
    posFromRelativePos(relativePos: IRelativePosition): number;
    /** SharedString.insertTextRelative / insertMarkerRelative */
    insertTextRelative(relativePos1: IRelativePosition, text: string, props?: PropertySet): MergeTreeOp | undefined;
    insertMarkerRelative(relativePos1: IRelativePosition, refType: number, props?: PropertySet): MergeTreeOp;
    /** PermutationVector.getAllocatedHandle (engines with caps.pcap > 0): the row's handle, allocated if it had none */
    getAllocatedHandle(pos: number): number;
    /** PermutationVector.getMaybeHandle: -2^31 (Handle.unallocated) when the row has none */
    getMaybeHandle(pos: number): number;
    /** HandleTable.snapshot() of this replica's PermutationVector */
    handleTable(): Int32Array;
    getLength(): number;
    /** SharedString.getText(start?, end?) of the local view */
    getText(start?: number, end?: number): string;
    /** SharedString.getTextWithPlaceholders / getTextRangeWithPlaceholders: non-text segments as " " */
    getTextWithPlaceholders(start?: number, end?: number): string;
    getLengthAt(refSeq: number, longClientId: string): number;
    /** MergeTreeTextHelper.getText(refSeq, clientId, placeholder, start, end); "*" throws (not modelled) */
    getTextAt(refSeq: number, longClientId: string, placeholder?: string, start?: number, end?: number): string;
    getContainingSegment(pos: number): { segment: SegmentHandle | undefined; offset: number | undefined };
    getPosition(segment: SegmentHandle): number;
    deltaEvents(): DeltaEvent[];
    /** every segment in walkAllSegments order, with its handle and local-view position */
    segments(): DecodedDump;
    /** Client.walkSegments (client.ts:276-285); splitRange needs caps.dcap, rcap or pcap > 0 */
    walkSegments<T>(handler: (segment: SegmentObject, pos: number, refSeq: number, clientId: string | undefined,
        start: number, end: number, accum?: T) => boolean, start?: number, end?: number, accum?: T, splitRange?: boolean): void;
    /** Client.getPropertiesAtPosition (client.ts:1011-1025) */
    getPropertiesAtPosition(pos: number): PropertySet | undefined;
    /** Client.getRangeExtentsOfPosition (client.ts:1026-1044) */
    getRangeExtentsOfPosition(pos: number): { posStart: number | undefined; posAfterEnd: number | undefined };
    /** MergeTree.resolveRemoteClientPosition (mergeTree.ts:2140-2160); throws "unsupported" where mt_engine.h says */
    resolveRemoteClientPosition(remoteClientPosition: number, remoteClientRefSeq: number, remoteLongClientId: string): number | undefined;
    /** Client.localTransaction (client.ts:961-981): every member a local op */
    localTransaction(groupOp: { type: 3; ops: MergeTreeOp[] }): void;
    /** Client.insertSegmentLocal for a segment spec (string, {text, props}, {marker, props}, [length, start]) */
    insertSegmentLocal(pos: number, spec: SegmentSpec | [number, number]): MergeTreeOp | undefined;
    /** Client.findTile (client.ts:1075-1078): the nearest Tile marker with the label, preceding startPos or after it */
    findTile(startPos: number | undefined, tileLabel: string, preceding?: boolean): { tile: SegmentObject; pos: number } | undefined;
    /** Client.getMarkerFromId (client.ts:312) */
    getMarkerFromId(id: string): SegmentObject | undefined;
    /** Client.annotateMarker (client.ts:143-154): the op with relative positions, or undefined */
    annotateMarker(marker: SegmentObject, props: PropertySet, combiningOp?: ICombiningOp): MergeTreeOp | undefined;
    /** PermutationVector.adjustPosition (permutationvector.ts:185-196) */
    adjustPosition(pos: number, fromSeq: number, longClientId: string): number | undefined;
    /** PermutationVector.handleToPosition (permutationvector.ts:198-253); localSeq defaults to the last local op's */
    handleToPosition(handle: number, localSeq?: number): number;
}

/** the Node-API addon itself (mt_napi.node) */
export declare const addon: { [fn: string]: (...args: unknown[]) => unknown };
